set -o pipefail
cd $GRAFT_REPO_ROOT
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 EXO_GRAPH_CHECK=0 timeout -k 10 300 python tools/packet_capture_check.py > gpurun_out/pc_check.json 2> gpurun_out/pc_check.err
rc=$?; cat gpurun_out/pc_check.json; tail -3 gpurun_out/pc_check.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/dp_layout_cost.py > gpurun_out/dp_layout_cost.json 2> gpurun_out/dp_layout_cost.err
rc=$?; cat gpurun_out/dp_layout_cost.json; exit $rc
