# round-3 validation on the GPU box: the full GPU test suite, then the
# round's rocprof evidence (profiles/collect.sh ${TAG:-r03b}) and the default bench
set -o pipefail
TAG=${1:-r03b}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_${TAG:-r03b}.log 2>&1 || { tail -40 gpurun_out/gpu_tests_${TAG:-r03b}.log; exit 1; }
tail -3 gpurun_out/gpu_tests_${TAG:-r03b}.log
bash profiles/collect.sh ${TAG:-r03b} > gpurun_out/collect_${TAG:-r03b}.log 2>&1 || { tail -20 gpurun_out/collect_${TAG:-r03b}.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/prof_${TAG:-r03b}/bench_default.log') if l.startswith('{\"metric')][-1])
print({k: d[k] for k in ('value','ms_per_step','grad_steps_per_sec')}); print(d['roofline']); print(d.get('valu_roofline'))"
