# fp32 select workgroup-cap: parity tests, then the fp32 loop and the td7 variants per cap
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_fused_gpu.py -k "select" > $O/tests.log 2>&1 || exit $?
for cap in ${CAPS:-0 128 64 0}; do
  EXO_SELECT_WG_CAP=$cap timeout -k 10 300 python3 bench.py --precision fp32 --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/f32_cap${cap}_$RANDOM.log 2>&1 || exit $?
done
