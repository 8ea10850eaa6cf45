# r05 A/B: the fp32 training loop (the reference's precision) with overlapped
# pairs: select_action's workgroup cap
set -e
mkdir -p gpurun_out/r05f32
A="--precision fp32 --steps 600 --warmup 60 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05f32/cap128_$i.log 2>&1
  EXO_LOOP_SELECT_CAP=0 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05f32/cap0_$i.log 2>&1
  EXO_LOOP_SELECT_CAP=64 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05f32/cap64_$i.log 2>&1
done
