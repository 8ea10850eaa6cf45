# packet-capture x select row-tile A/B (same box, default training bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp EXO_GRAPH_CHECK=0
O=gpurun_out/r03d_pc
mkdir -p $O
: > $O/ab.txt
for rep in 1 2 3; do
  for combo in "0 1" "1 1" "0 2" "1 2"; do
    set -- $combo
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$1 EXO_SELECT_RT=$2 timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('PC=$1 SELECT_RT=$2', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e6,3), 'M', round(d['grad_steps_per_sec']), d.get('finite'))" >> $O/ab.txt
  done
done
cat $O/ab.txt
