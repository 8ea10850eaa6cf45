# r05 A/B: encoder branch after the fixed pass with select_action capped at
# 128 / 96 workgroups per launch (EXO_LOOP_SELECT_CAP), default training window
set -e
mkdir -p gpurun_out/r05c2
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  EXO_ENC_AFTER=fixed timeout -k 10 200 python -u bench.py $A > gpurun_out/r05c2/encf_$i.log 2>&1
  EXO_ENC_AFTER=fixed EXO_LOOP_SELECT_CAP=128 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05c2/encf_cap128_$i.log 2>&1
  EXO_ENC_AFTER=fixed EXO_LOOP_SELECT_CAP=96 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05c2/encf_cap96_$i.log 2>&1
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05c2/base_$i.log 2>&1
done
