#!/bin/bash
# GPU box: capture fork/join audit tests + rollout graph tests, then the shipped-policy evaluation under multibody physics.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_capture_audit.py tests/test_rollout_gpu.py tests/test_metrics.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/audit_tests.log 2>&1 || exit $?
if [ -d policies ]; then
  timeout -k 10 400 python -u tools/eval_policies.py --physics multibody --out gpurun_out/eval_policies_multibody.json > gpurun_out/eval_policies_multibody.txt 2>&1 || exit $?
fi
