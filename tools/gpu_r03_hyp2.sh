set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u tools/eval_hypotheses.py --models shipped,swap_mag1_none --out gpurun_out/eval_hypotheses2.json > gpurun_out/eval_hypotheses2.txt 2>&1
rc=$?; grep -v "^  " gpurun_out/eval_hypotheses2.txt | tail -4; exit $rc
