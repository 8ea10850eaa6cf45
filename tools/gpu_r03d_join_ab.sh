# rollout-join placement A/B (same box), then a kernel trace with the join early
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_join
mkdir -p $O
: > $O/ab.txt
for rep in 1 2 3; do
  for j in 0 1; do
    EXO_ROLLOUT_EARLY_JOIN=$j timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('EARLY_JOIN=$j', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e6,3), 'M', round(d['grad_steps_per_sec']))" >> $O/ab.txt
  done
done
cat $O/ab.txt
OUT=$O/trace; mkdir -p $OUT
EXO_ROLLOUT_EARLY_JOIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $OUT/bench.log 2>&1 || exit $?
find $OUT -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
python3 tools/iter_timeline.py $OUT/kernel_trace.csv -v > $OUT/timeline.txt 2>&1
EXO_ROLLOUT_EARLY_JOIN=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_graph_order_gpu.py > $O/tests.log 2>&1; tail -3 $O/tests.log
