# which part of the default bench crashes under rocprofv3 --kernel-trace
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv"
B="python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline"
$P -d $O/main -o run -- $B --no-td7-variants --no-sync-rounds --no-reference-schedule > $O/main.log 2>&1 || exit $?
$P -d $O/var -o run -- $B --no-sync-rounds --no-reference-schedule > $O/var.log 2>&1 || exit $?
$P -d $O/sync -o run -- $B --no-td7-variants --no-reference-schedule > $O/sync.log 2>&1 || exit $?
$P -d $O/ref -o run -- $B --no-td7-variants --no-sync-rounds > $O/ref.log 2>&1
