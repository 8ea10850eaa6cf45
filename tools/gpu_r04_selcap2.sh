# loop select cap: fused tests, then bf16 / fp32 loops with EXO_LOOP_SELECT_CAP per arm
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_fused_gpu.py > $O/tests.log 2>&1 || exit $?
B="--steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds"
for arm in "bf16 unset" "bf16 128" "fp32 unset" "fp32 0" "bf16 unset" "bf16 128"; do
  set -- $arm
  if [ "$2" = unset ]; then
    timeout -k 10 300 python3 bench.py --precision $1 $B > $O/$1_$2_$RANDOM.log 2>&1 || exit $?
  else
    EXO_LOOP_SELECT_CAP=$2 timeout -k 10 300 python3 bench.py --precision $1 $B > $O/$1_$2_$RANDOM.log 2>&1 || exit $?
  fi
done
