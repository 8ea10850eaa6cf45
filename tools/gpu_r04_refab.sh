# reference-schedule rollout A/B: serial round graph (default) vs the
# branch-overlapped round graph with 16- and 32-row select tiles
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
B="--no-cpu-baseline --no-td7-variants --no-sync-rounds --steps 100 --warmup 20"
timeout -k 10 300 python3 bench.py $B > $O/serial.log 2>&1 || exit $?
EXO_REF_ROUND_GRAPH=1 timeout -k 10 300 python3 bench.py $B > $O/overlap_rt1.log 2>&1 || exit $?
EXO_REF_ROUND_GRAPH=1 EXO_SELECT_RT=2 timeout -k 10 300 python3 bench.py $B > $O/overlap_rt2.log 2>&1 || exit $?
EXO_SELECT_RT=2 timeout -k 10 300 python3 bench.py $B > $O/serial_rt2.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py $B > $O/serial2.log 2>&1
