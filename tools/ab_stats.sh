#!/bin/bash
# GPU box: rocprofv3 kernel stats of the training bench with switch $1 at 0 and 1
set -euo pipefail
VAR=${1:?switch variable}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 0 1; do
  OUT=gpurun_out/abstats_$v
  rm -rf $OUT && mkdir -p $OUT
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
      python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $OUT/bench.log 2>&1
  find $OUT -name "*kernel_stats.csv" -exec cp {} $OUT/stats.csv \;
  find $OUT -name "*kernel_trace.csv" -exec cp {} $OUT/trace.csv \;
done
