# fp32 training iteration (the per-layer path) under rocprofv3: kernel stats +
# trace for tools/iter_timeline.py; the bench line beside it.
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python3 bench.py --precision fp32 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule --steps 200 --warmup 30 > $O/bench_fp32.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o fp32 --output-format csv -- python3 bench.py --precision fp32 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule --steps 60 --warmup 20 > $O/prof_fp32.log 2>&1
