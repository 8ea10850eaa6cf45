set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_select_full_gpu.py tests/test_lap_gpu.py -v -s --timeout 120 --timeout-method thread > gpurun_out/t_sel.log 2>&1
rc=$?; tail -30 gpurun_out/t_sel.log; exit $rc
