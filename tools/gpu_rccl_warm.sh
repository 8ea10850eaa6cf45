# first RCCL process on a fresh box with a long warm-up, then a normal one
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
EXO_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29591 bench.py --steps 300 --warmup 60000 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/long_warm_first.log 2>&1 || exit $?
EXO_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29592 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/normal_second.log 2>&1
