#!/bin/bash
# GPU box: parity tests, then the round's rocprof evidence (profiles/collect.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
bash profiles/collect.sh ${1:-r01b}
