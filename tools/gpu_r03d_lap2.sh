# r03d: LAP store rank kernel with 16 rows per thread (A/B vs the previous lap.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_lap2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_lap_gpu.py tests/test_rollout_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
row() { python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('$1', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,3), 'M')"; }
: > $O/ab_wide.txt
for rep in 1 2; do
  for lib in libexo_amd.so libexo_amd_lapold.so; do
    EXO_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload wide --steps 20 --warmup 6 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    row "b128 $lib" >> $O/ab_wide.txt
  done
done
cat $O/ab_wide.txt
for lib in libexo_amd.so libexo_amd_lapold.so; do
  EXO_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/prof_$lib.log 2>&1 || exit 1
  f=$(find $O/prof_$lib -name "*kernel_stats.csv" | head -1)
  echo "== $lib" >> $O/lap_stats.txt
  grep -E "lap_store" $f >> $O/lap_stats.txt || true
done
cat $O/lap_stats.txt
