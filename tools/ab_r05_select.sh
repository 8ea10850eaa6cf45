# r05 A/B: select_action's CU footprint at the iteration start (default bench,
# training window only), two alternations per arm
set -e
mkdir -p gpurun_out/r05s
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05s/base_$i.log 2>&1
  EXO_SELECT_RT=2 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05s/rt2_$i.log 2>&1
  EXO_LOOP_SELECT_CAP=128 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05s/cap128_$i.log 2>&1
done
