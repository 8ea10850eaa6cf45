#!/bin/bash
# r06: the split select's zs half forked after the first iteration's env step
set -e
O=${1:-gpurun_out/r06sf}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rollout_gpu.py -k "overlapped_pairs" -m gpu > $O/tests.log 2>&1
bash tools/ab.sh $O/loop 3 "--steps 400 --warmup 50 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule" nosplit= env="EXO_SPLIT_SELECT=1 EXO_SPLIT_FORK=env" > $O/loop_summary.txt 2>&1
bash tools/ab.sh $O/loop32 2 "--steps 400 --warmup 50 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule --precision fp32" start= env="EXO_SPLIT_FORK=env" > $O/loop32_summary.txt 2>&1
