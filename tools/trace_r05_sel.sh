# r05: kernel traces of the training loop: rollout forked after the fixed pass,
# and select_action capped at 128 workgroups per launch
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/r05tr
A="--steps 300 --warmup 30 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
EXO_ROLLOUT_AFTER=fixed timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05tr/rollf -o run -- python3 bench.py $A > gpurun_out/r05tr/rollf.log 2>&1
EXO_ENC_AFTER=fixed EXO_LOOP_SELECT_CAP=128 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05tr/cap -o run -- python3 bench.py $A > gpurun_out/r05tr/cap.log 2>&1
