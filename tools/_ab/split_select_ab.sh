#!/bin/bash
# r06: select_action split at its zs image inside the overlapped pairs --
# bit-identity tests, then the training loop with and without (tools/ab.sh)
set -e
O=${1:-gpurun_out/r06ss}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fused_gpu.py tests/test_rollout_gpu.py -m gpu > $O/tests.log 2>&1
bash tools/ab.sh $O/loop 3 "--steps 400 --warmup 50 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule" split= nosplit="EXO_SPLIT_SELECT=0" > $O/loop_summary.txt 2>&1
bash tools/ab.sh $O/loop32 2 "--steps 400 --warmup 50 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule --precision fp32" split= nosplit="EXO_SPLIT_SELECT=0" > $O/loop32_summary.txt 2>&1
