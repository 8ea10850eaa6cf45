#!/bin/bash
# GPU box: whole -m gpu suite, then a kernel trace of the default training bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02b/train -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants > gpurun_out/prof_r02b_bench.log 2>&1
