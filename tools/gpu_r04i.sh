# round-4 GPU check i: hardware queues per process (graph branches -> queues) x target prefetch
set -o pipefail
O=gpurun_out/r04i2
mkdir -p $O
export PYTHONUNBUFFERED=1
B="--steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds"
for q in 2 3; do for pf in 0; do
  GPU_MAX_HW_QUEUES=$q EXO_TARGET_PREFETCH=$pf timeout -k 10 300 python3 bench.py $B > $O/bench_q${q}_pf${pf}.log 2>&1 || exit $?
done; done
