#!/bin/bash
# GPU box: A/B of an environment switch on the default training bench.
# usage: bash tools/gpu_ab_env.sh VAR "A B" [reps]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=$1; VALS=$2; REPS=${3:-2}
out=gpurun_out/ab_${VAR}.txt
: > $out
for rep in $(seq $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab_run.json')); print('$VAR=$v', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e6,3), 'M')" >> $out
  done
done
cat $out
