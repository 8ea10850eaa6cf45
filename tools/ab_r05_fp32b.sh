# r05 A/B: the fp32 loop with the critic-only iterations' select uncapped
# (default now) against the cap on every select
set -e
mkdir -p gpurun_out/r05f32b
A="--precision fp32 --steps 600 --warmup 60 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05f32b/capA_$i.log 2>&1
  EXO_LOOP_SELECT_CAP=128 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05f32b/cap128_$i.log 2>&1
  EXO_LOOP_SELECT_CAP_C=192 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05f32b/capC192_$i.log 2>&1
done
