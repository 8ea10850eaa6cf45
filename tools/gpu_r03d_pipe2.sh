# r03d: big forward GEMM with slices two ahead (TD7_BIG_PIPE2 build) vs the
# product library: per-GEMM timing, parity tests, wide iterations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_pipe2
mkdir -p $O
for lib in libexo_amd.so libexo_amd_pipe2.so; do
  echo "== $lib" >> $O/fwd_bench.txt
  EXO_AMD_LIB=$lib timeout -k 10 200 python3 tools/big_fwd_bench.py >> $O/fwd_bench.txt 2>/dev/null || exit 1
done
cat $O/fwd_bench.txt
EXO_AMD_LIB=libexo_amd_pipe2.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_td7_dense_gpu.py tests/test_configs_gpu.py tests/test_td7_full.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/ab_wide.txt
for rep in 1 2; do
  for lib in libexo_amd.so libexo_amd_pipe2.so; do
    EXO_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload wide --steps 20 --warmup 6 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('b128 $lib', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,3), 'M', d.get('critic_gemm_roofline',{}).get('frac'))" >> $O/ab_wide.txt
  done
done
for lib in libexo_amd.so libexo_amd_pipe2.so; do
  EXO_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload wide --batch 1024 --steps 12 --warmup 4 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('b1024 $lib', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,3), 'M', d.get('critic_gemm_roofline',{}).get('frac'))" >> $O/ab_wide.txt
done
cat $O/ab_wide.txt
