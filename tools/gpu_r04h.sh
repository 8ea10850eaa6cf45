# round-4 GPU check h: capture order x target prefetch A/B (+ bit-identity tests)
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_target_prefetch_gpu.py > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
B="--steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds"
for pf in 0 1; do for t in 0 1; do for a in 0 1; do
  EXO_TARGET_PREFETCH=$pf EXO_TD7_FIRST=$t EXO_ACTOR_FIRST=$a timeout -k 10 300 python3 bench.py $B > $O/bench_pf${pf}_t${t}_a${a}.log 2>&1 || exit $?
done; done; done
