# r03d: 16-bit AvgL1Norm outputs + 16-bit [a | zs] segments on the wide
# select chain, and the LAP store's single span propagation (A/B against the
# library with the previous lap.hip: EXO_AMD_LIB=libexo_amd_lapold.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_half3
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_lap_gpu.py tests/test_td7_dense_gpu.py tests/test_td7_ops_gpu.py tests/test_configs_gpu.py tests/test_td7_full.py tests/test_library.py tests/test_rollout_gpu.py tests/test_select_full_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
row() { python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('$1', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,3), 'M')"; }
: > $O/ab_wide.txt
for rep in 1 2; do
  for cfg in "libexo_amd.so 1" "libexo_amd_lapold.so 1" "libexo_amd.so 0"; do
    set -- $cfg
    EXO_AMD_LIB=$1 EXO_FWD_HALF=$2 timeout -k 10 300 python bench.py --workload wide --steps 20 --warmup 6 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    row "b128 $1 HALF=$2" >> $O/ab_wide.txt
  done
done
for lib in libexo_amd.so libexo_amd_lapold.so; do
  EXO_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload wide --batch 1024 --steps 12 --warmup 4 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
  row "b1024 $lib HALF=1" >> $O/ab_wide.txt
done
cat $O/ab_wide.txt
: > $O/ab_default.txt
for rep in 1 2; do
  for lib in libexo_amd.so libexo_amd_lapold.so; do
    EXO_AMD_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    row "default $lib" >> $O/ab_default.txt
  done
done
cat $O/ab_default.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --workload wide --steps 12 --warmup 6 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/wide_timeline.py $f > $O/timeline.txt
head -24 $O/timeline.txt
