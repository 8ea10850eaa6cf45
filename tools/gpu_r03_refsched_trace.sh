set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_rstrace
mkdir -p $O
for v in 1 0; do
  EXO_REF_ROUND_GRAPH=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rg$v -o run -- python3 tools/refsched_trace.py > $O/rg$v.log 2>&1 || { tail $O/rg$v.log; exit 1; }
done
ls $O/rg1 $O/rg0
