set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_ref_schedule_gpu.py tests/test_rollout_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_ref.log 2>&1
rc=$?
tail -30 gpurun_out/t_ref.log
exit $rc
