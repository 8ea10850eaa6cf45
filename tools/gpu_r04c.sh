# round-4 GPU check c: LAP kernels after the gather / span-propagation rework
# (bit-identity tests), the DR budget test, the default bench under the kernel
# tracer and alone, and configs[3] at budgets 0 / 96 / 256.
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
export PYTHONUNBUFFERED=1
T="tests/test_lap_gpu.py tests/test_trainer_fusion_gpu.py tests/test_step_budget_gpu.py tests/test_ref_schedule_gpu.py"
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $T > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o run -- \
    python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants > $O/bench_train_prof.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants > $O/bench_default.log 2>&1 && \
timeout -k 10 400 python3 bench.py --workload dr_sweep --step-budget 0 --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/bench_dr_b0.log 2>&1 && \
timeout -k 10 400 python3 bench.py --workload dr_sweep --step-budget 96 --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/bench_dr_b96.log 2>&1 && \
timeout -k 10 400 python3 bench.py --workload dr_sweep --step-budget 256 --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/bench_dr_b256.log 2>&1
