#!/bin/bash
# Same-box A/B of bench.py arms (run via gpurun).  Each arm is NAME=ENV where
# ENV is a space-separated list of VAR=VALUE settings ("" for the default);
# the arms alternate REPS times, each run under its own time limit, and every
# run's bench line lands in OUT/NAME_i.log.
#   usage: bash tools/ab.sh OUT REPS "BENCH ARGS" NAME=ENV [NAME=ENV ...]
#   e.g.   bash tools/ab.sh gpurun_out/ab 2 "--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants \
#              --no-sync-rounds --no-reference-schedule" base= pairs_off="EXO_OVERLAP_PAIRS=0"
# The r05 A/Bs (profiles/r05_sched/README.md) are arms of this script.
set -euo pipefail
OUT=$1; REPS=$2; ARGS=$3; shift 3
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  for arm in "$@"; do
    name=${arm%%=*}; vars=${arm#*=}
    env $vars timeout -k 10 300 python3 -u bench.py $ARGS > "$OUT/${name}_$i.log" 2>&1
  done
done
for f in "$OUT"/*.log; do
  python3 - "$f" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{"metric')]
print(sys.argv[1], json.loads(l[-1])["ms_per_step"] if l else "no line")
PY
done
