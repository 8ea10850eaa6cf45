set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_lap
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_lap_gpu.py tests/test_ref_schedule_gpu.py > $O/tests.log 2>&1; tail -2 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-td7-variants > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/run.log') if l.startswith('{\"metric')][-1]); r=d['reference_schedule']
print('ref-slots-v2', round(r['env_steps_per_sec']/1e6,3), 'M env-steps/s', round(r['ms_per_round'],2), 'ms/round', round(r['rollout_ms_per_round'],2), 'rollout ms', round(r['burst_ms_per_round'],2), 'burst ms', round(r['grad_steps_per_sec']), 'grad/s')" | tee -a $O/ab.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/refsched_trace.py > $O/p.log 2>&1 || exit 1
grep -h "lap_store_ref_slots\|lap_add_kernel\|lap_store_copy" $O/p/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
