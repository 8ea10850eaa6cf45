# configs[4] at batch 8 x 128: kernel trace, one iteration's timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_wide_tl
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --workload wide --steps 12 --warmup 6 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/wide_timeline.py $f > $O/timeline.txt
head -120 $O/timeline.txt
