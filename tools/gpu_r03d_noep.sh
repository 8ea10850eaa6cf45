#!/bin/bash
# GPU box: timing upper bound of removing the fused epilogue's ring drain
# (libexo_amd_noep.so: epilogue operand loads compiled out -- wrong numerics,
# timing only) against the product library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libexo_amd.so libexo_amd_noep.so; do
  echo "== $lib" >> gpurun_out/noep_fused_bench.txt
  EXO_AMD_LIB=$lib timeout -k 10 150 python -u tools/fused_bench.py >> gpurun_out/noep_fused_bench.txt 2>&1 || exit $?
done
bash tools/gpu_ab_lib.sh libexo_amd.so libexo_amd_noep.so 2
