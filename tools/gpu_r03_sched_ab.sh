# training-loop schedule A/B (same box): EXO_TD7_TARGET_ON_MAIN x EXO_PRIO_BRANCH_ALL,
# then the loop / capture / update parity tests with the defaults
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_sched
mkdir -p $O
: > $O/ab.txt
for rep in 1 2 3; do
  for combo in "0 1" "1 1" "0 0" "1 0"; do
    set -- $combo
    EXO_TD7_TARGET_ON_MAIN=$1 EXO_PRIO_BRANCH_ALL=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('TARGET_ON_MAIN=$1 PRIO_BRANCH_ALL=$2', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e6,3), 'M', round(d['grad_steps_per_sec']))" >> $O/ab.txt
  done
done
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_td7_full.py tests/test_ref_schedule_gpu.py tests/test_fused_gpu.py tests/test_packet_capture_gpu.py > $O/tests.log 2>&1; tail -3 $O/tests.log
