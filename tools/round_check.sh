#!/bin/bash
# End-of-round check on the GPU box: gpu tests, smoke, default + wide benches,
# rocprof kernel stats of the default bench and the env kernel, and the two
# PMC passes for the env kernel's HBM traffic.  Every GPU step has its own
# time limit and the steps are chained with && (stop at the first failure).
# usage (from the repo root, via gpurun): bash tools/round_check.sh TAG
set -o pipefail
TAG=${1:-r03f}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 &&
timeout -k 10 300 python bench.py --workload wide --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_wide.log 2>&1 &&
timeout -k 10 300 python bench.py --workload wide --batch 1024 --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_wide_b1024.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train_stats -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants > $O/bench_train_prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/env_stats -o run -- python3 bench.py --mode env --steps 300 --warmup 20 --no-cpu-baseline > $O/bench_env.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex exo_step --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --mode env --steps 50 --warmup 5 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex exo_step --output-format csv -d $O/pmc_write -o run -- python3 bench.py --mode env --steps 50 --warmup 5 --no-cpu-baseline > $O/pmc_write.log 2>&1
rc=$?
echo "round_check rc=$rc"
tail -2 $O/gpu_tests.log
exit $rc
