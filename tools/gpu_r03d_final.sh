# end-of-session check: the full GPU suite, smoke(), the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$O/bench_default.log') if l.startswith('{\"metric')][-1])
print({k: d[k] for k in ('value','ms_per_step','grad_steps_per_sec')}, d['roofline']['frac'], d['reference_schedule']['env_steps_per_sec'])"
