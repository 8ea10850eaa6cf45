set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_big2
mkdir -p $O
EXO_FWD_BIG=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_td7_dense_gpu.py -k "big_forward" > $O/tests2.log 2>&1; tail -2 $O/tests2.log
for v in 0 1 2; do EXO_FWD_BIG=$v timeout -k 10 200 python tools/big_fwd_bench.py > $O/bench_$v.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }; cat $O/bench_$v.json; done
