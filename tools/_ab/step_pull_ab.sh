#!/bin/bash
# exo_step_rp exchange forms: base library (parent commit) vs the product
# library with EXO_RP_GATHER=2 (LDS slots) and =3 (slots + DPP for r)
set -e
O=${1:-gpurun_out/r06p}; mkdir -p $O
for i in 1 2 3; do
  for arm in base g2 g3; do
    L=libexo_amd.so; G=2; [ $arm = base ] && L=libexo_amd_base.so; [ $arm = g3 ] && G=3
    EXO_RP_GATHER=$G EXO_AMD_LIB=$L timeout -k 10 180 python3 -u tools/step_ab.py $O/${arm}_rows_$i --rounds 10 > $O/${arm}_rows_$i.log 2>&1
    EXO_RP_GATHER=$G EXO_AMD_LIB=$L timeout -k 10 180 python3 -u tools/step_ab.py $O/${arm}_shared_$i --rounds 10 --variant rows_shared > $O/${arm}_shared_$i.log 2>&1
  done
done
for v in rows shared; do for a in g2 g3; do
  python3 tools/step_ab.py --compare $O/base_${v}_1_traj.json $O/${a}_${v}_1_traj.json > $O/compare_${a}_${v}.log 2>&1 || true
done; done
EXO_RP_GATHER=3 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_env_gpu.py tests/test_rhs_exchange_gpu.py -m gpu > $O/env_tests_g3.log 2>&1
