# r05 A/B: encoder branch after the fixed pass (EXO_ENC_AFTER=fixed) with the
# rollout branch at the iteration start or after the fixed pass too
# (EXO_ROLLOUT_AFTER=fixed), default training bench window
set -e
mkdir -p gpurun_out/r05e2
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05e2/base_$i.log 2>&1
  EXO_ENC_AFTER=fixed timeout -k 10 200 python -u bench.py $A > gpurun_out/r05e2/encf_$i.log 2>&1
  EXO_ENC_AFTER=fixed EXO_ROLLOUT_AFTER=fixed timeout -k 10 200 python -u bench.py $A > gpurun_out/r05e2/encf_rollf_$i.log 2>&1
  EXO_ROLLOUT_AFTER=fixed timeout -k 10 200 python -u bench.py $A > gpurun_out/r05e2/rollf_$i.log 2>&1
done
