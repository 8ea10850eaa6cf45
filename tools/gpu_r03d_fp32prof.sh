# fp32 TD7 (the reference's precision, per-layer kernels): kernel-time split
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_fp32
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --precision fp32 --steps 100 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -30 $f | cut -d, -f1-4 | cut -c1-170
grep '^{"metric' $O/prof.log | cut -c1-300
