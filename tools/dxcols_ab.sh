set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_td7_dense_gpu.py tests/test_td7_ops_gpu.py tests/test_graph_order_gpu.py tests/test_rollout_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dxcols_tests.log 2>&1 || exit $?
for i in 1 2 3; do
  EXO_TD7_DX_COLS=0 timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/ab_off_$i.json 2>gpurun_out/ab_err.log || exit $?
  EXO_TD7_DX_COLS=1 timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/ab_on_$i.json 2>gpurun_out/ab_err.log || exit $?
done
