#!/bin/bash
# GPU box: configs[4] (wide) iteration time under the trainer's schedule switches
set -o pipefail
mkdir -p gpurun_out/ws
export TMPDIR=/tmp
out=gpurun_out/ws/summary.txt
: > $out
for sw in NONE=1 EXO_TD7_OVERLAP=0 EXO_ROLLOUT_OVERLAP=0 EXO_TD7_ACTOR_BRANCH=0 EXO_TD7_TARGET_BRANCH=0 EXO_SAMPLE_PREFETCH=0 EXO_PRIO_BRANCH=0; do
  env $sw timeout -k 10 300 python3 bench.py --workload wide --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/ws/b.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/ws/b.log').read().strip().splitlines()[-1]); print('$sw', round(d['value']), round(d['ms_per_step'],4))" | tee -a $out
done
