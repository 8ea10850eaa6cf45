# env step kernel: same-box A/B of two library builds (rocprof, env mode and
# the training loop's rows_shared shape), then the env parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_env_ab
mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for lib in libexo_amd_pre.so libexo_amd.so; do
    d=$O/${lib%.so}_$rep
    EXO_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --mode env --steps 300 --warmup 20 --no-cpu-baseline > $d.log 2>&1 || { tail $d.log; exit 1; }
    python3 -c "
import csv
for r in csv.DictReader(open('$d/run_kernel_stats.csv')):
    if 'exo_step' in r['Name']: print('$lib rep $rep', r['Name'][40:75], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')" >> $O/ab.txt
  done
done
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_env_gpu.py tests/test_rhs_exchange_gpu.py tests/test_multibody_gpu.py tests/test_rollout_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1; tail -3 $O/tests.log
