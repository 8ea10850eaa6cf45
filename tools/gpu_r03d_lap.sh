# r03d LAP kernels: parity tests, same-box A/B against the previous LAP kernels,
# kernel stats of both; then the data-parallel layout on RCCL at world 1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_lap
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_lap_gpu.py tests/test_rollout_gpu.py tests/test_ref_schedule_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
: > $O/ab.txt
for rep in 1 2 3; do
  for lib in libexo_amd_prev.so libexo_amd.so; do
    EXO_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/run.json 2> $O/run.err || { tail $O/run.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/run.json') if l.startswith('{\"metric')][-1]); print('$lib', round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e6,3), 'M', round(d['grad_steps_per_sec']))" >> $O/ab.txt
  done
done
cat $O/ab.txt
for lib in libexo_amd_prev.so libexo_amd.so; do
  EXO_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$lib -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-td7-variants --no-reference-schedule > $O/prof_$lib.log 2>&1 || exit 1
  f=$(find $O/prof_$lib -name "*kernel_stats.csv" | head -1); grep -i "lap_" $f | cut -d, -f1-8 >> $O/lap_stats_$lib.csv
done
EXO_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 200 --warmup 20 --no-cpu-baseline \
    --no-td7-variants --no-reference-schedule > $O/rccl_world1.json 2> $O/rccl_world1.err || { tail $O/rccl_world1.err; exit 1; }
grep '^{"metric' $O/rccl_world1.json | cut -c1-400
