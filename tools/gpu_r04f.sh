# round-4 GPU check f: cross-iteration target prefetch -- capture check, the
# bit-identity tests, the tests it touches, then the bench A/B and a kernel
# trace of the prefetching loop.
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 python3 tools/seg_bisect.py 128 512 1 > $O/seg_bisect.log 2>&1 || exit $?
T="tests/test_target_prefetch_gpu.py tests/test_rollout_gpu.py tests/test_trainer_fusion_gpu.py tests/test_dp_gpu.py tests/test_configs_gpu.py tests/test_capture_audit.py"
timeout -k 10 800 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu $T > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
B="--steps 300 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds"
timeout -k 10 300 python3 bench.py $B > $O/bench_prefetch.log 2>&1 && \
EXO_TARGET_PREFETCH=0 timeout -k 10 300 python3 bench.py $B > $O/bench_noprefetch.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o run -- \
    python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule --no-sync-rounds > $O/bench_train_prof.log 2>&1
