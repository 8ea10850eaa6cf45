#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/<round>_*.md / .json.

usage: python profiles/summarize.py ROUND STATS_DIR [PMC_FETCH_DIR PMC_WRITE_DIR] [--bytes-per-launch B]

* STATS_DIR: `rocprofv3 --kernel-trace --stats --output-format csv -o run`
  output (run_kernel_stats.csv) of the bench command.
* PMC dirs: `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes (one
  counter per pass, --kernel-include-regex exo_step).  FETCH_SIZE/WRITE_SIZE
  are in KiB; per MI355X_MICROARCH.md (HBM section) gfx950 FETCH_SIZE tallies
  half of the bytes of coalesced streaming reads, so reads are doubled.
"""
import csv
import json
import os
import sys

import numpy as np


def kernel_stats(d):
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))
    out = []
    for r in rows:
        out.append(dict(name=r["Name"], calls=int(r["Calls"]), total_ms=float(r["TotalDurationNs"]) / 1e6,
                        avg_us=float(r["AverageNs"]) / 1e3, min_us=float(r["MinNs"]) / 1e3,
                        max_us=float(r["MaxNs"]) / 1e3, pct=float(r["Percentage"])))
    return out


def pmc(d, counter, match="exo_step"):
    rows = [r for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv")))
            if match in r["Kernel_Name"] and r["Counter_Name"] == counter]
    v = np.array([float(r["Counter_Value"]) for r in rows])
    return dict(counter=counter, launches=int(v.size), mean_kib=float(v.mean()), median_kib=float(np.median(v)))


def main():
    args = sys.argv[1:]
    bpl = None
    if "--bytes-per-launch" in args:
        i = args.index("--bytes-per-launch")
        bpl = float(args[i + 1])
        del args[i:i + 2]
    rnd, stats = args[0], args[1]
    here = os.path.dirname(os.path.abspath(__file__))
    ks = kernel_stats(stats)
    res = {"round": rnd, "kernels": ks[:40]}
    lines = [f"# rocprofv3 kernel summary ({rnd})", "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for k in ks[:25]:
        lines.append(f"| `{k['name'][:90]}` | {k['calls']} | {k['total_ms']:.2f} | {k['avg_us']:.1f} | {k['pct']:.1f} |")
    if len(args) >= 4:
        f, w = pmc(args[2], "FETCH_SIZE"), pmc(args[3], "WRITE_SIZE")
        traffic = (2 * f["median_kib"] + w["median_kib"]) * 1024
        res["pmc_exo_step"] = dict(fetch=f, write=w, traffic_bytes_per_launch=traffic,
                                   correction="reads x2 (gfx950 FETCH_SIZE half-tally), KiB x 1024",
                                   algorithmic_bytes_per_launch=bpl)
        lines += ["", "## exo_step_kernel HBM traffic (PMC, per launch)", "",
                  f"- FETCH_SIZE median {f['median_kib']:.1f} KiB over {f['launches']} launches (x2 gfx950 correction)",
                  f"- WRITE_SIZE median {w['median_kib']:.1f} KiB",
                  f"- traffic = (2*FETCH + WRITE) * 1024 = {traffic / 1e6:.3f} MB per launch"]
        if bpl:
            lines.append(f"- algorithmic bytes per launch = {bpl / 1e6:.3f} MB -> traffic/algorithmic = {traffic / bpl:.2f}")
    open(os.path.join(here, f"{rnd}_rocprof_summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump(res, open(os.path.join(here, f"{rnd}_rocprof_summary.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
