# r05: full GPU test suite, then the default bench line and the configs[3] /
# configs[4] lines (each step under its own time limit; stop at the first failure)
set -e
mkdir -p gpurun_out/r05f
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05f/tests.log 2>&1
timeout -k 10 500 python3 bench.py > gpurun_out/r05f/bench_default.log 2>&1
timeout -k 10 300 python3 bench.py --workload dr_sweep --steps 200 --warmup 20 --no-cpu-baseline --no-reference-schedule > gpurun_out/r05f/bench_dr.log 2>&1
timeout -k 10 300 python3 bench.py --workload wide --steps 60 --warmup 10 --no-cpu-baseline --no-reference-schedule > gpurun_out/r05f/bench_wide.log 2>&1
