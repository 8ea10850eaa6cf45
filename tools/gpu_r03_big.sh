set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_big
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_td7_dense_gpu.py -k "big_forward or lds_forward or cat" > $O/tests.log 2>&1; tail -3 $O/tests.log
EXO_FWD_BIG=0 timeout -k 10 200 python tools/big_fwd_bench.py > $O/bench_old.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 200 python tools/big_fwd_bench.py > $O/bench_new.json 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench_old.json $O/bench_new.json
for rep in 1 2; do
  for big in 0 1; do
    EXO_FWD_BIG=$big timeout -k 10 300 python bench.py --workload wide --steps 60 --warmup 15 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/wide_$big.log 2>&1 || { tail $O/wide_$big.log; exit 1; }
    python3 -c "
import json
l=[x for x in open('$O/wide_$big.log') if x.startswith('{\"metric\"')][-1]; d=json.loads(l)
print('wide EXO_FWD_BIG=$big', round(d['ms_per_step'],4), 'ms', round(d['value']/1e6,3), 'M')"
  done
done
