# round-4 GPU check (reusable): the given test files, then the default bench
# with any A/B environment passed in AB ("VAR=a VAR=b"; one bench per value).
# usage: T="tests/x.py ..." AB="EXO_X=0 EXO_X=1" bash tools/gpu_r04_ab.sh OUTDIR [bench args]
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ -n "$T" ]; then
  timeout -k 10 800 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu $T > $O/tests.log 2>&1
  rc=$?
  [ $rc -le 1 ] || exit $rc
fi
for kv in ${AB:-NONE=1}; do
  env $kv timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-td7-variants "$@" > $O/bench_${kv}.log 2>&1 || exit $?
done
