#!/bin/bash
# GPU box: kernel trace of the default training bench (no variant sub-runs) for tools/iter_timeline.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > gpurun_out/tl.log 2>&1 || exit $?
python3 tools/iter_timeline.py gpurun_out/tl/run_kernel_trace.csv -v > gpurun_out/timeline.txt 2>&1
