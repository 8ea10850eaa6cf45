set -o pipefail
mkdir -p gpurun_out/pc
export EXO_GRAPH_CHECK=0
for i in 1 2; do
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/pc/b0_$i.json 2>/dev/null || exit $?
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/pc/b1_$i.json 2>/dev/null || exit $?
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 python -u -m pytest tests/test_rollout_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pc/rollout_pc1.log 2>&1
echo rollout_rc=$? >> gpurun_out/pc/rollout_pc1.log
