# round-4 GPU check d: async (auto-reset) episodes -- parity tests, then the
# training bench sync vs async at configs[1] and configs[3] (budgets 0 / 96 / 160).
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
export PYTHONUNBUFFERED=1
T="tests/test_async_episodes_gpu.py tests/test_rollout_gpu.py tests/test_step_budget_gpu.py"
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $T > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
B="--steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule"
timeout -k 10 300 python3 bench.py $B --episodes async > $O/bench_c1_async.log 2>&1 && \
timeout -k 10 300 python3 bench.py $B --episodes sync > $O/bench_c1_sync.log 2>&1 && \
timeout -k 10 400 python3 bench.py $B --workload dr_sweep --episodes async --step-budget 0 > $O/bench_dr_async_b0.log 2>&1 && \
timeout -k 10 400 python3 bench.py $B --workload dr_sweep --episodes async --step-budget 96 > $O/bench_dr_async_b96.log 2>&1 && \
timeout -k 10 400 python3 bench.py $B --workload dr_sweep --episodes async --step-budget 160 > $O/bench_dr_async_b160.log 2>&1
