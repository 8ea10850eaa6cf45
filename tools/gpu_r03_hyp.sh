set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -x -q -k tremor_model --timeout 120 --timeout-method thread > gpurun_out/t_trem.log 2>&1 || { tail -30 gpurun_out/t_trem.log; exit 1; }
tail -2 gpurun_out/t_trem.log
timeout -k 10 900 python -u tools/eval_hypotheses.py --out gpurun_out/eval_hypotheses.json > gpurun_out/eval_hypotheses.txt 2>&1
rc=$?; grep -v "^  " gpurun_out/eval_hypotheses.txt | tail -12; exit $rc
