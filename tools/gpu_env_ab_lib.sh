#!/bin/bash
# GPU box: exo_step kernel time (env-only bench under rocprof kernel stats) for two library builds, alternated.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/env_ab_lib.txt
: > $out
for rep in 1 2; do
  for lib in $1 $2; do
    rm -rf gpurun_out/envab
    EXO_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/envab -o run -- python3 bench.py --mode env --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/envab.log 2>&1 || exit $?
    python3 -c "
import csv; r=[x for x in csv.DictReader(open('gpurun_out/envab/run_kernel_stats.csv')) if 'exo_step' in x['Name']]
print('$lib', [(x['Calls'], round(float(x['AverageNs'])/1e3,2), round(float(x['MinNs'])/1e3,2)) for x in r])" >> $out
  done
done
cat $out
