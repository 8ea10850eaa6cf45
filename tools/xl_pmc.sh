#!/bin/bash
# PMC passes (one rocprofv3 run each) over tools/xl_pmc.py's
# dense_fwd_xl8_kernel launches; run via gpurun from the repo root.
set -euo pipefail
OUT=gpurun_out/r05_xlpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
R="--kernel-include-regex dense_fwd_xl8 --output-format csv"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS $R -d $OUT/p1 -o run -- python3 tools/xl_pmc.py > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUSY_max $R -d $OUT/p2 -o run -- python3 tools/xl_pmc.py > $OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE $R -d $OUT/p3 -o run -- python3 tools/xl_pmc.py > $OUT/p3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE $R -d $OUT/p4 -o run -- python3 tools/xl_pmc.py > $OUT/p4.log 2>&1
