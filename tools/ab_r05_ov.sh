# r05 A/B: overlapped pairs (EXO_OVERLAP_PAIRS=1) and select_action's shape
# inside them (32-row tiles / 128-workgroup cap), default training window
set -e
mkdir -p gpurun_out/r05ov3
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  EXO_OVERLAP_PAIRS=1 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05ov3/ov_$i.log 2>&1
  EXO_OVERLAP_PAIRS=1 EXO_SELECT_RT=2 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05ov3/ov_rt2_$i.log 2>&1
  EXO_OVERLAP_PAIRS=1 EXO_LOOP_SELECT_CAP=128 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05ov3/ov_cap128_$i.log 2>&1
  EXO_OVERLAP_PAIRS=1 EXO_ENC_AFTER=0 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05ov3/ov_enc0_$i.log 2>&1
done
