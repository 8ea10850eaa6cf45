#!/bin/bash
# Same-box A/B of exo_step_rp: the product library against libexo_amd_base.so
# (built from the parent commit's sources), alternating processes; outputs
# digested for a bit-for-bit check; phase stamps of both (stamps libraries)
# and of the EXO_STAMPS_MEMWAIT diagnostic build; the env GPU tests.
#   usage (on the GPU box): bash tools/step_ab.sh OUT [REPS]
set -e
O=${1:-gpurun_out/r06s}; REPS=${2:-3}; mkdir -p $O
for i in $(seq 1 $REPS); do
  for lib in base new; do
    L=libexo_amd.so; [ $lib = base ] && L=libexo_amd_base.so
    EXO_AMD_LIB=$L timeout -k 10 180 python3 -u tools/step_ab.py $O/${lib}_rows_$i --rounds 10 > $O/${lib}_rows_$i.log 2>&1
    EXO_AMD_LIB=$L timeout -k 10 180 python3 -u tools/step_ab.py $O/${lib}_shared_$i --rounds 10 --variant rows_shared > $O/${lib}_shared_$i.log 2>&1
  done
done
python3 tools/step_ab.py --compare $O/base_rows_1_traj.json $O/new_rows_1_traj.json > $O/compare_rows.log 2>&1 || true
python3 tools/step_ab.py --compare $O/base_shared_1_traj.json $O/new_shared_1_traj.json > $O/compare_shared.log 2>&1 || true
for s in base new mw; do
  L=libexo_amd_stamps_$s.so; [ $s = new ] && L=libexo_amd_stamps.so
  EXO_AMD_LIB=$L timeout -k 10 180 python3 -u profiles/stamps_rp.py > $O/stamps_$s.json 2>$O/stamps_$s.err
done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_env_gpu.py tests/test_rhs_exchange_gpu.py tests/test_async_episodes_gpu.py tests/test_step_budget_gpu.py tests/test_multibody_gpu.py -m gpu > $O/env_tests.log 2>&1
