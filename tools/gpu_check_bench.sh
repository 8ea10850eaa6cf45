#!/bin/bash
# GPU box: the whole -m gpu suite, then 3 default training benches (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/cb_*.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cb_tests.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/cb_$i.json 2>gpurun_out/cb_err.log || exit $?
done
for f in gpurun_out/cb_*.json; do
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'], 4), d['weights_finite'])"
done | tee gpurun_out/cb_summary.txt
