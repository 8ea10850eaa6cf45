#!/bin/bash
# GPU box: (1) the data-parallel layout on RCCL at world 1 (torchrun, one rank,
# EXO_FORCE_DIST=1: process group, flat-bucket all-reduces between the graph
# segments, MAX reductions, replica checksum all_gather), (2) a kernel trace of
# the default training bench for the iteration timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
EXO_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 200 --warmup 20 --no-cpu-baseline \
    --no-td7-variants --no-reference-schedule > gpurun_out/rccl_world1.json 2> gpurun_out/rccl_world1.err || exit $?
bash tools/trace_iter.sh default || exit $?
python3 tools/iter_timeline.py gpurun_out/trace_default/kernel_trace.csv -v > gpurun_out/trace_default/timeline.txt 2>&1
