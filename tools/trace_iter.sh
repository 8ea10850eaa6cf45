#!/bin/bash
# Kernel trace of the training bench (timeline analysis: tools/iter_timeline.py)
# usage: [EXO_...=...] bash tools/trace_iter.sh [tag]
set -euo pipefail
OUT=gpurun_out/trace${1:+_$1}
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline > $OUT/bench.log 2>&1
find $OUT -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
