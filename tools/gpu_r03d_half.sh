# r03d: 16-bit activations on the wide inference chain (EXO_FWD_HALF)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_half2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_td7_dense_gpu.py tests/test_td7_ops_gpu.py tests/test_configs_gpu.py tests/test_td7_full.py tests/test_library.py tests/test_rollout_gpu.py tests/test_select_full_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1; do
  echo "== EXO_FWD_HALF=$v" >> $O/fwd_bench.txt
  EXO_FWD_HALF=$v timeout -k 10 200 python3 tools/big_fwd_bench.py >> $O/fwd_bench.txt 2>/dev/null || exit 1
done
cat $O/fwd_bench.txt
: > $O/ab_wide.txt
for rep in 1 2; do
  for v in 0 1; do
    EXO_FWD_HALF=$v timeout -k 10 300 python bench.py --workload wide --steps 20 --warmup 6 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('b128 EXO_FWD_HALF=$v', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,3), 'M')" >> $O/ab_wide.txt
  done
done
for v in 0 1; do
  EXO_FWD_HALF=$v timeout -k 10 300 python bench.py --workload wide --batch 1024 --steps 12 --warmup 4 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('b1024 EXO_FWD_HALF=$v', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,3), 'M')" >> $O/ab_wide.txt
done
cat $O/ab_wide.txt
