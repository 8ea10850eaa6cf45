# RCCL world-1 main loop at different step counts (no other bench phases)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
p=29570
for sw in "300 40" "400 50" "200 250"; do
  set -- $sw
  p=$((p+1))
  EXO_FORCE_DIST=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=$p bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/bench_$1_$2.log 2>&1 || exit $?
done
timeout -k 10 400 python3 bench.py --steps 400 --warmup 50 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/single_400_50.log 2>&1
