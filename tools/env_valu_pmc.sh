#!/bin/bash
# fp64 VALU instruction counts of the env step kernel (one rocprofv3 --pmc pass)
set -o pipefail
mkdir -p gpurun_out/valu
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES --kernel-include-regex exo_step --output-format csv -d gpurun_out/valu -o run -- python3 bench.py --mode env --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/valu/bench.log 2>&1
