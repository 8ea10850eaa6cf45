# same-box A/B of two builds of the library on the wide configuration, then
# the dense-kernel parity tests with the new one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_wide_ab
mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for lib in libexo_amd_pre.so libexo_amd.so; do
    EXO_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload wide --steps 60 --warmup 15 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
    python3 -c "
import json
l=[x for x in open('$O/run.log') if x.startswith('{\"metric\"')][-1]; d=json.loads(l)
print('$lib', round(d['ms_per_step'],4), 'ms')" >> $O/ab.txt
  done
done
cat $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload wide --steps 60 --warmup 15 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/prof.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_td7_dense_gpu.py tests/test_td7_full.py tests/test_configs_gpu.py tests/test_td7_ops_gpu.py > $O/tests.log 2>&1; tail -3 $O/tests.log
