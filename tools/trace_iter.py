"""Break one steady-state training iteration of a rocprofv3 kernel trace into
kernel classes: python tools/trace_iter.py gpurun_out/prof_X/train/run_kernel_trace.csv"""
import csv
import re
import sys
from collections import defaultdict


def classify(n):
    base = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if base.startswith("td7f::"):
        return "td7 fused (HIP)"
    if "adam_multi" in base:
        return "Adam (HIP)"
    if base.startswith("lap_"):
        return "LAP (HIP)"
    if "dense_" in n.split("(")[0] or "(anonymous namespace)::dense" in n:
        return "td7_dense (HIP)"
    if "exo_step" in n:
        return "env step (HIP)"
    if n.startswith("lap_") or "lap_" in n.split("(")[0]:
        return "LAP (HIP)"
    if "dense_gemm" in n:
        return "td7_dense (HIP)"
    if "avgl1" in n:
        return "AvgL1Norm (HIP)"
    if n.startswith("Cijk") or "gemm" in n.lower() or "Tensile" in n:
        return "GEMM (hipBLASLt)"
    if "FusedOpti" in n or "multi_tensor_apply" in n:
        return "Adam"
    if "reduce_kernel" in n:
        return "torch reduce"
    if "CatArray" in n:
        return "torch cat"
    if "fillBuffer" in n or "FillFunctor" in n:
        return "fill/memset"
    if "index" in n.lower() or "gather" in n.lower() or "scatter" in n.lower():
        return "torch index"
    if "elementwise" in n or "Functor" in n:
        return "torch elementwise"
    return "other"


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "exo_step" in r["Kernel_Name"]]
    # a steady-state iteration: between two env-step launches late in the run (train loop, not kernel_timing)
    k = len(starts) // 3
    a, b = starts[k], starts[k + 1]
    it = rows[a:b]
    t0, t1 = int(it[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in it)
    cls = defaultdict(lambda: [0, 0.0])
    for r in it:
        c = classify(r["Kernel_Name"])
        cls[c][0] += 1
        cls[c][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"iteration: {len(it)} kernels, wall {(t1 - t0) / 1e3:.1f} us, kernel-busy {busy / 1e3:.1f} us")
    for c, (n, us) in sorted(cls.items(), key=lambda x: -x[1][1]):
        print(f"  {c:22s} {n:4d} kernels {us:8.1f} us  avg {us / n:6.2f}")
    if "-v" in sys.argv:
        for r in it:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"{d:7.2f}  {r['Kernel_Name'][:120]}")


if __name__ == "__main__":
    main(sys.argv[1])
