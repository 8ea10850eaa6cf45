#!/bin/bash
# GPU box: exchange-form + env parity tests on the current library, exo_step A/B
# (base vs current, env bench under rocprof), then the fp64 VALU PMC pass
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rhs_exchange_gpu.py tests/test_env_gpu.py tests/test_rollout_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tq_tests.log 2>&1 || exit $?
bash tools/gpu_env_ab_lib.sh libexo_amd_base.so libexo_amd.so && cp gpurun_out/env_ab_lib.txt gpurun_out/ab_torque_lds.txt || exit $?
bash tools/env_valu_pmc.sh
