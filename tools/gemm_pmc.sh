#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/gpmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex dense_fwd --output-format csv -d gpurun_out/gpmc/p1 -o run -- python3 tools/gemm_pmc.py > gpurun_out/gpmc/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex dense_fwd --output-format csv -d gpurun_out/gpmc/p2 -o run -- python3 tools/gemm_pmc.py > gpurun_out/gpmc/p2.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --kernel-include-regex dense_fwd --output-format csv -d gpurun_out/gpmc/t -o run -- python3 tools/gemm_pmc.py > gpurun_out/gpmc/t.log 2>&1
