# r05 A/B with overlapped pairs: the env step's shape in the training loop
# (rows_shared 32 envs / 512 threads vs the 256-thread default shape)
set -e
mkdir -p gpurun_out/r05sh
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05sh/shared_$i.log 2>&1
  EXO_TRAIN_STEP_SHARED=0 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05sh/default_$i.log 2>&1
done
