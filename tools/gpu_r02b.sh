#!/bin/bash
# GPU box: whole -m gpu suite, then the round's profile evidence (profiles/collect.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1 || exit $?
bash profiles/collect.sh "${1:-r02b}"
if [ -d policies ]; then
  timeout -k 10 300 python -u tools/eval_policies.py --out gpurun_out/eval_policies_ideal.json > gpurun_out/eval_policies_ideal.txt 2>&1 || exit $?
fi
