# RCCL world-1 main loop, repeated fresh processes, hardware-queue count A/B
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
p=29580
for q in 4 8 4 8 4 8 4 8; do
  p=$((p+1))
  GPU_MAX_HW_QUEUES=$q EXO_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=$p bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/q${q}_$p.log 2>&1 || exit $?
done
