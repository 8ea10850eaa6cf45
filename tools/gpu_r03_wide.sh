# configs[4] (wide TD7, 65,536 envs, fp16): same-box A/B of the round-1 tree
# (ab_r01 = commit cfb99c1, its own bench.py and library) against the current
# tree, each under the rocprofv3 kernel tracer and plain; then the current tree
# at batch 8 x 1,024.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_wide
mkdir -p $O
W="--workload wide --steps 60 --warmup 15 --no-cpu-baseline"
for rep in 1 2; do
  (cd ab_r01 && timeout -k 10 300 python bench.py $W > ../$O/r01_plain_$rep.log 2>&1) || { tail $O/r01_plain_$rep.log; exit 1; }
  timeout -k 10 300 python bench.py $W --no-td7-variants --no-reference-schedule > $O/cur_plain_$rep.log 2>&1 || { tail $O/cur_plain_$rep.log; exit 1; }
done
(cd ab_r01 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../$O/r01_prof -o run -- python3 bench.py $W > ../$O/r01_prof.log 2>&1) || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cur_prof -o run -- python3 bench.py $W --no-td7-variants --no-reference-schedule > $O/cur_prof.log 2>&1 || exit 1
timeout -k 10 400 python bench.py $W --batch 1024 --no-td7-variants --no-reference-schedule > $O/cur_b1024.log 2>&1 || { tail $O/cur_b1024.log; exit 1; }
for f in $O/*_plain_*.log $O/cur_b1024.log; do python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{\"metric\"')][-1]; d=json.loads(l)
print('$f', round(d['ms_per_step'],4), round(d['value']/1e6,3), d.get('grad_steps_per_sec'))"; done
