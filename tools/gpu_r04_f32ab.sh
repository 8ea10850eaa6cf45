# fp32 fused training-loop schedule A/B (one bench per AB value)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for kv in NONE=1 EXO_TD7_TARGET_ON_MAIN=1 EXO_ENC_SPLIT=1 EXO_PRIO_BRANCH_ALL=1 NONE=2; do
  env $kv timeout -k 10 300 python3 bench.py --precision fp32 --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/f32_${kv}.log 2>&1 || exit $?
done
