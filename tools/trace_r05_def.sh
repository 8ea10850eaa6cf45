# r05: the default bench line, then a kernel trace of the default training loop
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/r05d
timeout -k 10 500 python3 bench.py > gpurun_out/r05d/bench_default.log 2>&1
A="--steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05d/tr -o run -- python3 bench.py $A > gpurun_out/r05d/tr.log 2>&1
