set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_lap_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_lap.log 2>&1 || { tail -30 gpurun_out/t_lap.log; exit 1; }
tail -3 gpurun_out/t_lap.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_r03a.log 2>&1 || { tail -30 gpurun_out/bench_r03a.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_r03a.log').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step','grad_steps_per_sec')}); print(json.dumps(d['reference_schedule'], indent=1)); print(d['td7_variants'])"
