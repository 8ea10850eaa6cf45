#!/bin/bash
# GPU box: A/B of two builds of the native library on the default training bench.
# usage: bash tools/gpu_ab_lib.sh LIB_A LIB_B [reps]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/ab_lib.txt
: > $out
for rep in $(seq ${3:-2}); do
  for lib in $1 $2; do
    EXO_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab_run.json')); print('$lib', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e6,3), 'M')" >> $out
  done
done
cat $out
