# timing-only experiment: the big forward GEMM with W's (SMALL_B) or X's
# (SMALL_A) footprint shrunk to 256 rows -- what each operand's traffic costs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_traffic
mkdir -p $O
for lib in libexo_amd.so libexo_amd_SMALL_B.so libexo_amd_SMALL_A.so; do
  echo "== $lib" >> $O/fwd_bench.txt
  EXO_AMD_LIB=$lib timeout -k 10 200 python3 tools/big_fwd_bench.py >> $O/fwd_bench.txt 2>/dev/null || exit 1
done
cat $O/fwd_bench.txt
