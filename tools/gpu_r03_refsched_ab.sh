# reference-schedule sub-line: round graph (overlapped replay inserts) vs per-step graphs, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_refsched
mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for v in 0 1; do
    EXO_REF_ROUND_GRAPH=$v timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-td7-variants > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/run.log') if l.startswith('{\"metric')][-1]); r=d['reference_schedule']
print('EXO_REF_ROUND_GRAPH=$v', round(r['env_steps_per_sec']/1e6,3), 'M env-steps/s', round(r['ms_per_round'],2), 'ms/round', round(r['rollout_ms_per_round'],2), 'rollout ms', round(r['burst_ms_per_round'],2), 'burst ms', round(r['grad_steps_per_sec']), 'grad/s')" >> $O/ab.txt
  done
done
cat $O/ab.txt
