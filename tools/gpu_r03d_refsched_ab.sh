# reference-schedule sub-line: round graph (inserts beside the next select) x
# select row tile (32 rows per workgroup leaves half the CUs to the inserts)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_refsched
mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for combo in "0 1" "1 1" "0 2" "1 2"; do
    set -- $combo
    EXO_REF_ROUND_GRAPH=$1 EXO_SELECT_RT=$2 timeout -k 10 300 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-td7-variants > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/run.log') if l.startswith('{\"metric')][-1]); r=d['reference_schedule']
print('ROUND_GRAPH=$1 SELECT_RT=$2', round(r['env_steps_per_sec']/1e6,3), 'M env-steps/s', round(r['ms_per_round'],2), 'ms/round', round(r['rollout_ms_per_round'],2), 'rollout ms', round(r['burst_ms_per_round'],2), 'burst ms', round(r['grad_steps_per_sec']), 'grad/s')" >> $O/ab.txt
  done
done
cat $O/ab.txt
