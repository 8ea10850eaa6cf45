# round-4 GPU check: the new/affected GPU tests, the RCCL world-1 bench, the
# default bench and the host-vs-GPU iteration split.  A step that does not end
# in a pass or an ordinary test failure (exit 0 / 1) stops the script.
set -o pipefail
mkdir -p gpurun_out/r04a
export PYTHONUNBUFFERED=1
T="tests/test_noise_schedule_gpu.py tests/test_lap_gpu.py tests/test_step_budget_gpu.py tests/test_encoder_split_gpu.py tests/test_metrics.py tests/test_env_gpu.py tests/test_rhs_exchange_gpu.py tests/test_dp_gpu.py tests/test_ref_schedule_gpu.py tests/test_fused_gpu.py tests/test_td7_full.py tests/test_trainer_fusion_gpu.py tests/test_rollout_gpu.py"
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu $T > gpurun_out/r04a/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
EXO_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29513 bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants > gpurun_out/r04a/bench_rccl_w1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants > gpurun_out/r04a/bench_default.log 2>&1 && \
timeout -k 10 200 python tools/host_bound.py > gpurun_out/r04a/host_bound.log 2>&1
