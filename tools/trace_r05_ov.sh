# r05: kernel trace of the training loop with overlapped pairs (EXO_OVERLAP_PAIRS=1)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/r05tr
A="--steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
EXO_OVERLAP_PAIRS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05tr/ov -o run -- python3 bench.py $A > gpurun_out/r05tr/ov.log 2>&1
