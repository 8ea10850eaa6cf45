#!/bin/bash
# GPU box: per-kernel times of the fused passes (product library) and stamps (diagnostic library)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
EXO_FUSED_NOSTAMPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof2 -o run -- python3 tools/fused_stamps_train.py > gpurun_out/fprof2.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/fused_stamps_train.py > gpurun_out/fused_stamps_train.txt 2>&1 || exit $?
timeout -k 10 150 python -u tools/fused_stamps.py > gpurun_out/fused_stamps.txt 2>&1 || exit $?
