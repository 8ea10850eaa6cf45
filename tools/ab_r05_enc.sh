# r05 A/B: when the encoder update's branch starts (EXO_ENC_AFTER), default
# training bench window, alternating arms
set -e
mkdir -p gpurun_out/r05e
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05e/base_$i.log 2>&1
  EXO_ENC_AFTER=fixed timeout -k 10 200 python -u bench.py $A > gpurun_out/r05e/fixed_$i.log 2>&1
  EXO_ENC_AFTER=target timeout -k 10 200 python -u bench.py $A > gpurun_out/r05e/target_$i.log 2>&1
done
