#!/bin/bash
# GPU box: the whole -m gpu suite on the current library, exo_step A/Bs (base vs
# current) at 4,096 envs (row-parallel kernel) and 65,536 envs (two-lane kernel),
# then the round's rocprof evidence under tag $1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
bash tools/gpu_env_ab_lib.sh libexo_amd_base.so libexo_amd.so && cp gpurun_out/env_ab_lib.txt gpurun_out/ab_fastpow.txt || exit $?
out=gpurun_out/ab_fastpow_65536.txt
: > $out
for rep in 1 2; do
  for lib in libexo_amd_base.so libexo_amd.so; do
    rm -rf gpurun_out/envab
    EXO_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/envab -o run -- python3 bench.py --mode env --envs 65536 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/envab.log 2>&1 || exit $?
    python3 -c "
import csv; r=[x for x in csv.DictReader(open('gpurun_out/envab/run_kernel_stats.csv')) if 'exo_step' in x['Name']]
print('$lib', [(x['Name'][:40], x['Calls'], round(float(x['AverageNs'])/1e3,2), round(float(x['MinNs'])/1e3,2)) for x in r])" >> $out
  done
done
cat $out
bash profiles/collect.sh ${1:-r02f}
