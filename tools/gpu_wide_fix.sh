#!/bin/bash
# GPU box: the configs[4] wide workload after the step-variant threshold, plus the configs tests
set -o pipefail
mkdir -p gpurun_out/wl
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py tests/test_rollout_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wl/wide_fix_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --workload wide --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/wl/bench_wide_fix.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --workload dr_sweep --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/wl/bench_dr_sweep2.log 2>&1
