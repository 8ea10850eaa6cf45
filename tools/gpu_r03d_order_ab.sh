# dispatch-order A/B (same box): EXO_UPDATE_FIRST x EXO_SELECT_RT, then the
# loop / capture parity tests with EXO_UPDATE_FIRST=1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_order
mkdir -p $O
: > $O/ab.txt
for rep in 1 2 3; do
  for combo in "0 1" "1 1" "0 2" "1 2"; do
    set -- $combo
    EXO_UPDATE_FIRST=$1 EXO_SELECT_RT=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('UPDATE_FIRST=$1 SELECT_RT=$2', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e6,3), 'M', round(d['grad_steps_per_sec']))" >> $O/ab.txt
  done
done
cat $O/ab.txt
EXO_UPDATE_FIRST=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_capture_audit.py tests/test_graph_order_gpu.py tests/test_trainer_fusion_gpu.py > $O/tests.log 2>&1; tail -3 $O/tests.log
