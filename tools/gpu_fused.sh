#!/bin/bash
# GPU box: the fused-TD7 parity tests, the TD7 tests they feed, the per-pass timing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_td7_full.py tests/test_td7.py tests/test_rollout_gpu.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?
timeout -k 10 120 python -u tools/fused_bench.py > gpurun_out/fused_bench.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants > gpurun_out/fused_train_bench.json 2> gpurun_out/fused_train_bench.err || exit $?
timeout -k 10 150 python -u tools/fused_stamps_train.py > gpurun_out/fused_stamps_train.txt 2>&1 || exit $?
exit $rc
