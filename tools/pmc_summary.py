"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one or more passes).

usage: python tools/pmc_summary.py OUTDIR [kernel-regex]  -> a markdown table
of every counter's mean per dispatch for each kernel matching the regex, plus
derived ratios where their counters are present."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(root, pat):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch]
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if not re.search(pat, k):
                    continue
                per[(row["Dispatch_Id"], k, row["Counter_Name"])] += float(row["Counter_Value"])
        for (d, k, c), v in per.items():
            vals[k][c].append(v)
    return vals


def short(k):
    m = re.search(r"td7f::(\w+)<([^>]*)>", k)
    return f"{m.group(1)}<{m.group(2)}>" if m else k[:60]


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "."
    vals = load(root, pat)
    counters = sorted({c for k in vals for c in vals[k]})
    print("| kernel | dispatches | " + " | ".join(counters) + " |")
    print("|---|---|" + "---|" * len(counters))
    for k in sorted(vals):
        n = max(len(v) for v in vals[k].values())
        cells = [f"{sum(vals[k][c]) / len(vals[k][c]):.4g}" if vals[k].get(c) else "" for c in counters]
        print(f"| `{short(k)}` | {n} | " + " | ".join(cells) + " |")
    print()
    print("| kernel | MFMA busy / (busy CU cycles x 4 SIMD) | wait-inst / wave-cycles | wait-any / wave-cycles | "
          "LDS conflict / LDS active | L2 hit |")
    print("|---|---|---|---|---|---|")
    for k in sorted(vals):
        m = {c: sum(v) / len(v) for c, v in vals[k].items() if v}

        def r(a, b, scale=1.0):
            return f"{m[a] / (m[b] * scale):.3f}" if a in m and b in m and m[b] else ""
        hit = (f"{m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}"
               if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m else "")
        print(f"| `{short(k)}` | {r('SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_BUSY_CU_CYCLES', 4.0)} | "
              f"{r('SQ_WAIT_INST_ANY', 'SQ_WAVE_CYCLES')} | {r('SQ_WAIT_ANY', 'SQ_WAVE_CYCLES')} | "
              f"{r('SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE')} | {hit} |")


if __name__ == "__main__":
    main()
