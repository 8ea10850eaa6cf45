set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_dr
timeout -k 10 300 python tools/rk45_hist.py --workload dr_sweep > gpurun_out/r03_dr/rk45_hist_dr_sweep.json 2> gpurun_out/r03_dr/rk45_hist.err || { tail gpurun_out/r03_dr/rk45_hist.err; exit 1; }
timeout -k 10 300 python tools/rk45_hist.py --workload configs1 > gpurun_out/r03_dr/rk45_hist_configs1.json 2>> gpurun_out/r03_dr/rk45_hist.err || exit 1
timeout -k 10 400 python bench.py --workload dr_sweep --steps 344 --warmup 30 --no-cpu-baseline > gpurun_out/r03_dr/bench_dr_sweep.log 2>&1 || { tail gpurun_out/r03_dr/bench_dr_sweep.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_dr/train -o run -- python3 bench.py --workload dr_sweep --steps 344 --warmup 30 --no-cpu-baseline --no-reference-schedule > gpurun_out/r03_dr/bench_dr_sweep_prof.log 2>&1 || exit 1
cat gpurun_out/r03_dr/rk45_hist_dr_sweep.json | head -c 1500; echo
grep exo_step gpurun_out/r03_dr/train/run_kernel_stats.csv | cut -c1-160
