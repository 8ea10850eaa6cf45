# configs[4] bench lines with the current library: batch 8 x 128 and 8 x 1,024
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_wide_lines
mkdir -p $O
timeout -k 10 400 python bench.py --workload wide --no-cpu-baseline > $O/bench_wide_b128.log 2>&1 || { tail $O/bench_wide_b128.log; exit 1; }
timeout -k 10 600 python bench.py --workload wide --batch 1024 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_wide_b1024.log 2>&1 || { tail $O/bench_wide_b1024.log; exit 1; }
for f in $O/bench_wide_b128.log $O/bench_wide_b1024.log; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{\"metric\"')][-1]; d=json.loads(l)
print('$f', round(d['ms_per_step'],4), 'ms', round(d['value']/1e6,3), 'M env-steps/s', round(d['grad_steps_per_sec'],1), 'grad/s', d['td7_roofline']['achieved'], d['critic_gemm_roofline'])"; done
