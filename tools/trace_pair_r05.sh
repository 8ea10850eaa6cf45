# r05: kernel traces of the default training loop with and without pair graphs
# (EXO_PAIR_GRAPHS=1: two iterations per graph launch) for the timeline of the
# graph boundary (tools/iter_timeline.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/r05pair
A="--steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05pair/base -o run -- python3 bench.py $A > gpurun_out/r05pair/base.log 2>&1
EXO_PAIR_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05pair/pair -o run -- python3 bench.py $A > gpurun_out/r05pair/pair.log 2>&1
