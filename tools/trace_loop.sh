#!/bin/bash
# rocprofv3 kernel trace of the training loop (run via gpurun), for the
# iteration timelines of DESIGN.md 4 ("The training iteration's schedule").
#   usage: bash tools/trace_loop.sh OUT ["VAR=VALUE ..."] ["BENCH ARGS"]
# The environment settings are exported before rocprofv3 starts (the program
# itself follows --, never env / bash -c).
set -euo pipefail
OUT=$1; VARS=${2:-}; ARGS=${3:-"--steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"}
mkdir -p "$OUT"
for v in $VARS; do export "$v"; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run -- python3 bench.py $ARGS > "$OUT/tr.log" 2>&1
