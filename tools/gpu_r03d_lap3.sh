# r03d: LAP store rank kernel, rows per thread 4 (<= 16,384 envs) / 16 (above)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_lap3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_lap_gpu.py tests/test_rollout_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/lap_stats.txt
for lib in libexo_amd.so libexo_amd_lapold.so; do
  EXO_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/prof_$lib.log 2>&1 || exit 1
  f=$(find $O/prof_$lib -name "*kernel_stats.csv" | head -1)
  echo "== default $lib" >> $O/lap_stats.txt
  grep -E "lap_store" $f >> $O/lap_stats.txt || true
  EXO_AMD_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wprof_$lib -o run -- python3 bench.py --workload wide --steps 12 --warmup 6 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/wprof_$lib.log 2>&1 || exit 1
  f=$(find $O/wprof_$lib -name "*kernel_stats.csv" | head -1)
  echo "== wide $lib" >> $O/lap_stats.txt
  grep -E "lap_store" $f >> $O/lap_stats.txt || true
done
cat $O/lap_stats.txt
