set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_b1024
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload wide --batch 1024 --steps 30 --warmup 10 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/prof.log 2>&1 || exit 1
head -25 $O/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
