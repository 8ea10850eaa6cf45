#!/bin/bash
# A/B of the 16-bit large-layer forward kernels (EXO_FWD_XL=v, td7_dense.hip:
# 0 dense_fwd_big_kernel, 1 dense_fwd_xl_kernel, 2 the default
# dense_fwd_xl8_kernel) on tools/wide_gemm_compare.py, then the XL parity
# test under each value named in TEST (run via gpurun from the repo root).
#   VARS="0 2" TEST="1 2" bash tools/xl_ab.sh
OUT=gpurun_out/r05x
mkdir -p $OUT
for v in ${VARS:-0 2}; do
  EXO_FWD_XL=$v timeout -k 10 150 python -u tools/wide_gemm_compare.py > $OUT/cmp_v$v.log 2>&1 || exit 1
done
for v in ${TEST:-}; do
  EXO_FWD_XL=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_td7_dense_gpu.py -k xl_forward > $OUT/xltest$v.log 2>&1 || exit 1
done
