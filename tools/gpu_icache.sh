#!/bin/bash
# GPU box: list the SQ/SQC counters, then instruction-cache and wait counters of the fused gradient passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_VALU --kernel-include-regex td7f --output-format csv -d gpurun_out/pmc_icache -o run -- python3 tools/fused_stamps_train.py > gpurun_out/pmc_icache.log 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex td7f --output-format csv -d gpurun_out/pmc_wait -o run -- python3 tools/fused_stamps_train.py > gpurun_out/pmc_wait.log 2>&1 || true
