# r05: capture-order experiments inside the overlapped pairs -- tests with the
# flags on, then a same-box A/B of the default training window
set -e
mkdir -p gpurun_out/r05o
T="tests/test_fused_gpu.py::test_fused_trainer_graph_replay_equals_eager tests/test_rollout_gpu.py"
EXO_TRAIN_FIRST=1 EXO_PAIR_CRITIC_AFTER_SELECT=1 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread $T > gpurun_out/r05o/tests.log 2>&1
A="--steps 1000 --warmup 100 --no-cpu-baseline --no-td7-variants --no-sync-rounds --no-reference-schedule"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r05o/base_$i.log 2>&1
  EXO_TRAIN_FIRST=1 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05o/tf_$i.log 2>&1
  EXO_PAIR_CRITIC_AFTER_SELECT=1 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05o/cas_$i.log 2>&1
  EXO_TRAIN_FIRST=1 EXO_PAIR_CRITIC_AFTER_SELECT=1 timeout -k 10 200 python -u bench.py $A > gpurun_out/r05o/both_$i.log 2>&1
done
