set -e
mkdir -p gpurun_out/r05q
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05q/shared1_$i.log 2>&1
  EXO_TRAIN_STEP_SHARED=0 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05q/shared0_$i.log 2>&1
done
