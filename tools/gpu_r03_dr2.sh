set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_dr
timeout -k 10 300 python tools/rk45_hist.py --workload dr_sweep --launches 20 --eager-launches 30 > gpurun_out/r03_dr/rk45_eager_dr_sweep.json 2> gpurun_out/r03_dr/rk45_eager.err || { tail gpurun_out/r03_dr/rk45_eager.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r03_dr/rk45_eager_dr_sweep.json'))
print(d['per_launch_max'], d['graph_act_abs_mean'][:5])
for e in d['eager_launches']: print(e)
"
