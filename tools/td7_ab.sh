#!/bin/bash
# GPU box: TD7 kernel/op tests, then an interleaved A/B of the training bench
# with the switch $1 (an EXO_* environment variable) at 0 and 1.
# usage: bash tools/td7_ab.sh EXO_TD7_CAT
set -o pipefail
VAR=${1:?switch variable}
mkdir -p gpurun_out
rm -f gpurun_out/ab_*.json
timeout -k 10 300 python -u -m pytest tests/test_device_rng_gpu.py tests/test_td7_dense_gpu.py tests/test_td7_ops_gpu.py tests/test_graph_order_gpu.py tests/test_rollout_gpu.py tests/test_lap_gpu.py tests/test_td7.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || exit $?
for i in 1 2 3; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/ab_${v}_$i.json 2>gpurun_out/ab_err.log || exit $?
  done
done
for f in gpurun_out/ab_*_*.json; do
  python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'], 4))"
done | tee gpurun_out/ab_summary.txt
