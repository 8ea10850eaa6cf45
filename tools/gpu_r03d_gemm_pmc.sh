# PMC passes (one per run, SQ/TCC limits respected) over the wide forward GEMM
# of tools/big_fwd_bench.py (dense_fwd_big_kernel): where a wave's cycles go
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d_gemm_pmc
mkdir -p $O
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU" \
            "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex dense_fwd_big --output-format csv -d $O/p$i -o run -- python3 tools/big_fwd_bench.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  f=$(find $O/p$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$pass" >> $O/summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    name = r.get("Kernel_Name", r.get("Kernel-Name", ""))[:70]
    grid = r.get("Grid_Size", "")
    agg[(name, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (n, g), cs in agg.items():
    print(n, "grid", g, {c: round(sum(v) / len(v)) for c, v in cs.items()})
PY
done
cat $O/summary.txt
