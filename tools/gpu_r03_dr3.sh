set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_dr3
timeout -k 10 400 python bench.py --workload dr_sweep --steps 344 --warmup 30 --no-cpu-baseline --no-reference-schedule > gpurun_out/r03_dr3/bench_dr_sweep.log 2>&1 || { tail gpurun_out/r03_dr3/bench_dr_sweep.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_dr3/train -o run -- python3 bench.py --workload dr_sweep --steps 344 --warmup 30 --no-cpu-baseline --no-reference-schedule > gpurun_out/r03_dr3/bench_dr_sweep_prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03_dr3/bench_default.log 2>&1 || { tail gpurun_out/r03_dr3/bench_default.log; exit 1; }
python - <<'PY'
import json
for f in ("bench_dr_sweep.log", "bench_dr_sweep_prof.log", "bench_default.log"):
    b = json.loads(open("gpurun_out/r03_dr3/" + f).read().strip().splitlines()[-1])
    r = b["roofline"]
    print(f, b["value"], b["ms_per_step"], r["avg_kernel_ms"], r.get("window_step_clock"), r.get("loop_workload", {}).get("avg_kernel_ms"), b.get("grad_steps_per_sec"))
PY
