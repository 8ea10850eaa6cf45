#!/bin/bash
# GPU box: the other BASELINE workloads (configs[3] DR sweep, configs[4] wide) with
# rocprof kernel stats of the wide one
set -o pipefail
mkdir -p gpurun_out/wl
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload dr_sweep --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/wl/bench_dr_sweep.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --workload wide --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/wl/bench_wide.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wl/wide -o run -- python3 bench.py --workload wide --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/wl/bench_wide_prof.log 2>&1
