#!/bin/bash
# GPU box: rocprof kernel stats of the default training bench under two values
# of an environment switch (same box, same run).
# usage: bash tools/gpu_ab_env_stats.sh VAR "A B"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=$1; VALS=$2
for v in $VALS; do
  rm -rf gpurun_out/abst_$v
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abst_$v -o run -- \
      python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants > gpurun_out/abst_$v.log 2>&1 || exit $?
done
