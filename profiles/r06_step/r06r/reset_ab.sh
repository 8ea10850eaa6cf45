#!/bin/bash
# exo_env.hip's scratch-free invert: step/reset timing + trajectory digests
# (tools/step_ab.py) and the training loop (tools/ab.sh), base vs product
set -e
O=${1:-gpurun_out/r06r}; mkdir -p $O
for i in 1 2; do
  for lib in base new; do
    L=libexo_amd.so; [ $lib = base ] && L=libexo_amd_base.so
    EXO_AMD_LIB=$L timeout -k 10 180 python3 -u tools/step_ab.py $O/${lib}_rows_$i --rounds 5 > $O/${lib}_rows_$i.log 2>&1
  done
done
python3 tools/step_ab.py --compare $O/base_rows_1_traj.json $O/new_rows_1_traj.json > $O/compare_rows.log 2>&1 || true
bash tools/ab.sh $O/loop 3 "--steps 400 --warmup 50 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule" base="EXO_AMD_LIB=libexo_amd_base.so" new= > $O/loop_summary.txt 2>&1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_env_gpu.py tests/test_async_episodes_gpu.py -m gpu > $O/env_tests.log 2>&1
