# RCCL world-1 (EXO_FORCE_DIST=1 under torchrun) bench, one run per AB value
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
p=29540
for kv in $AB; do
  p=$((p+1))
  env $kv EXO_FORCE_DIST=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=$p bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/bench_${kv}.log 2>&1 || exit $?
done
