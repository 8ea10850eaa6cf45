#!/bin/bash
# GPU box: exchange-form tests (incl. the folded-I^-1 form 3), env tests under form 3,
# then A/B of forms 2 / 3: env kernel under rocprof and the training loop
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rhs_exchange_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fold_tests.log 2>&1 || exit $?
EXO_RP_GATHER=3 timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_rollout_gpu.py tests/test_multibody_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread >> gpurun_out/fold_tests.log 2>&1 || exit $?
out=gpurun_out/ab_fold.txt
: > $out
for rep in 1 2; do
  for g in 2 3; do
    rm -rf gpurun_out/envab
    EXO_RP_GATHER=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/envab -o run -- python3 bench.py --mode env --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/envab.log 2>&1 || exit $?
    python3 -c "
import csv; r=[x for x in csv.DictReader(open('gpurun_out/envab/run_kernel_stats.csv')) if 'exo_step' in x['Name']]
print('env GATHER=$g', [(x['Calls'], round(float(x['AverageNs'])/1e3,2), round(float(x['MinNs'])/1e3,2)) for x in r])" >> $out
  done
done
for rep in 1 2; do
  for g in 2 3; do
    EXO_RP_GATHER=$g timeout -k 10 200 python3 bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/fold_bench.json 2>gpurun_out/fold_bench_err.log || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/fold_bench.json').read().strip().splitlines()[-1]); print('train GATHER=$g', round(d['value']), round(d['ms_per_step'],4), d['roofline']['avg_kernel_ms'], d['roofline']['training_loop_variant']['avg_kernel_ms_alone'])" >> $out
  done
done
cat $out
