# first RCCL process on a fresh box with a longer warm-up (arg 2), then a normal one
set -o pipefail
O=gpurun_out/$1
W=${2:-2000}
mkdir -p $O
EXO_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29595 bench.py --steps 300 --warmup $W --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/warm${W}_first.log 2>&1 || exit $?
EXO_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29596 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/normal_second.log 2>&1
