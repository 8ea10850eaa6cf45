# fp32 fused path on the GPU: its parity tests first, then the td7 variant
# lines (fp32 per-layer vs fp32 fused vs bf16 alias) from a short bench.
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_fused_gpu.py "tests/test_td7_full.py::test_three_train_steps_at_bench_shape_gpu_fused_fp32" "tests/test_td7_full.py::test_three_train_steps_at_bench_shape_gpu" > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-sync-rounds --no-reference-schedule --steps 50 --warmup 20 > $O/bench.log 2>&1
