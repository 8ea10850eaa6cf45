# round-4 GPU check b: the budget/env/rollout tests after the solver-failure
# change, the kernel trace of the default bench (iteration + reference-schedule
# timelines), the A/B of the fused insert and the encoder split, and the
# configs[3] budgeted bench with its RK45 histogram.  A step that does not end
# in a pass or an ordinary test failure (exit 0 / 1) stops the script.
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
export PYTHONUNBUFFERED=1
T="tests/test_step_budget_gpu.py tests/test_env_gpu.py tests/test_rollout_gpu.py tests/test_rhs_exchange_gpu.py"
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $T > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o run -- \
    python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants > $O/bench_train_prof.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants > $O/bench_ab_default.log 2>&1 && \
EXO_REF_INSERT_FUSED=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants > $O/bench_ab_nofusedins.log 2>&1 && \
EXO_ENC_SPLIT=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/bench_ab_noencsplit.log 2>&1 && \
timeout -k 10 400 python3 bench.py --workload dr_sweep --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/bench_dr.log 2>&1 && \
timeout -k 10 300 python3 tools/rk45_hist.py --workload dr_sweep --budget 160 --launches 60 > $O/rk45_hist_dr_b160.json 2> $O/rk45_hist_dr_b160.err
