#!/bin/bash
# GPU box: rocprofv3 kernel stats of the wide TD7 configuration (configs[4])
set -euo pipefail
OUT=gpurun_out/wide_stats
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --workload wide --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1
