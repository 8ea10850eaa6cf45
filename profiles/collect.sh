#!/bin/bash
# Collect the round's rocprofv3 evidence on the GPU box (run via gpurun):
#   kernel stats of the default training bench, of the env-only bench, and the
#   FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) for the exo_step kernel,
#   then the default bench (CPU baseline included) and configs[3] plain.
# usage: bash profiles/collect.sh TAG
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# (r04: the whole default bench -- main loop, td7 variants, sync rounds and the
# reference schedule, ~10 graph-replayed trainers in one process -- segfaults
# inside CUDAGraph::replay under the kernel tracer, every phase alone does not
# (profiles/r04pc2_raw); the traced run is the main loop + reference schedule)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/train -o run -- \
    python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants --no-sync-rounds > $OUT/bench_train.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/env -o run -- \
    python3 bench.py --mode env --steps 300 --warmup 20 --no-cpu-baseline > $OUT/bench_env.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex exo_step --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 bench.py --mode env --steps 100 --warmup 10 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex exo_step --output-format csv -d $OUT/pmc_write -o run -- \
    python3 bench.py --mode env --steps 100 --warmup 10 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench_default.log 2>&1
timeout -k 10 400 python3 bench.py --workload dr_sweep --steps 200 --warmup 20 --no-cpu-baseline --no-reference-schedule > $OUT/bench_dr.log 2>&1
find $OUT -name "*.csv" | head -50
