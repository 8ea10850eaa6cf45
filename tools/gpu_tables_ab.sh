#!/bin/bash
# GPU box: env parity + exchange-form tests on the current library, then A/B
# (libexo_amd_base.so vs the current library): env kernel
# under rocprof, and the training loop
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rhs_exchange_gpu.py tests/test_env_gpu.py tests/test_rollout_gpu.py tests/test_multibody_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tb_tests.log 2>&1 || exit $?
bash tools/gpu_env_ab_lib.sh libexo_amd_base.so libexo_amd.so && cp gpurun_out/env_ab_lib.txt gpurun_out/ab_tables.txt || exit $?
for rep in 1 2; do
  for lib in libexo_amd_base.so libexo_amd.so; do
    EXO_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/tb_bench.json 2>gpurun_out/tb_bench_err.log || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/tb_bench.json').read().strip().splitlines()[-1]); print('train $lib', round(d['value']), round(d['ms_per_step'],4), d['roofline']['avg_kernel_ms'], d['roofline']['training_loop_variant']['avg_kernel_ms_alone'])" >> gpurun_out/ab_tables.txt
  done
done
cat gpurun_out/ab_tables.txt
