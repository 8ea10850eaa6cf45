# round-4 GPU check e: async episodes (reset after the final solve, compacted
# reset list), DP tests, the default bench (async + sync comparison +
# reference schedule), configs[3] default, and select RT=2 A/B.
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
export PYTHONUNBUFFERED=1
T="tests/test_async_episodes_gpu.py tests/test_dp_gpu.py tests/test_env_gpu.py"
timeout -k 10 800 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu $T > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants > $O/bench_default.log 2>&1 && \
EXO_SELECT_RT=2 timeout -k 10 300 python3 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/bench_select_rt2.log 2>&1 && \
timeout -k 10 400 python3 bench.py --workload dr_sweep --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/bench_dr.log 2>&1
