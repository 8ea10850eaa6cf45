# The RCCL world-1 in-graph layout in fresh processes (run via gpurun): the
# default training bench under EXO_FORCE_DIST=1 (no launcher: the env://
# rendezvous variables set here), the first RCCL process of the box first,
# then per-step host times of a later process (tools/rccl_step_times.py).
set -o pipefail
OUT=gpurun_out/${1:-r05rccl4}
mkdir -p $OUT
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 EXO_FORCE_DIST=1
ARGS="--no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds"
MASTER_PORT=29631 timeout -k 10 300 python3 bench.py $ARGS > $OUT/bench_p1.log 2>&1 &&
MASTER_PORT=29632 timeout -k 10 300 python3 bench.py $ARGS > $OUT/bench_p2.log 2>&1 &&
MASTER_PORT=29633 timeout -k 10 300 python3 tools/rccl_step_times.py 800 > $OUT/steps_p3.log 2>&1
