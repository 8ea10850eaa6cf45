#!/bin/bash
# GPU box: env parity tests, then exo_step_rp A/B: DPP gather vs LDS permutes (env-only bench, rocprof kernel stats).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_multibody_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/rp_tests.log 2>&1 || exit $?
for g in 0 0; do
  EXO_RP_GATHER=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_ab_$g -o run -- python3 bench.py --mode env --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/rp_ab_$g.log 2>&1 || exit $?
  python3 -c "
import csv; r=[x for x in csv.DictReader(open('gpurun_out/rp_ab_$g/run_kernel_stats.csv')) if 'exo_step' in x['Name']]
print('gather=$g', [(x['Name'][:40], x['Calls'], round(float(x['AverageNs'])/1e3,2)) for x in r])" >> gpurun_out/rp_ab.txt
done
