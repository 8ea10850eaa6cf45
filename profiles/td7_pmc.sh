#!/bin/bash
# Hardware counters of the fused TD7 passes in the training loop (run via
# gpurun): two rocprofv3 --pmc passes (separate runs; SQ <= 8, TCC <= 4,
# TA <= 2, GRBM <= 2 per pass) over a short default training bench, counters
# collected for the td7f:: kernels only.  usage: bash profiles/td7_pmc.sh TAG
set -euo pipefail
TAG=${1:-r05}
OUT=gpurun_out/td7pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS="--steps 60 --warmup 10 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT \
    --kernel-include-regex 'td7f::' --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA \
    --kernel-include-regex 'td7f::' --output-format csv -d $OUT/p2 -o run -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --kernel-include-regex 'td7f::' --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
find $OUT -name "*.csv" | head -20
