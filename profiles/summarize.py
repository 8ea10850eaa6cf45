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


def iteration_classes(stats_dir):
    """Kernel classes of one steady-state training iteration (tools/trace_iter.py)."""
    trace = os.path.join(stats_dir, "run_kernel_trace.csv")
    if not os.path.exists(trace):
        return None, []
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import trace_iter
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "exo_step" in r["Kernel_Name"]]
    # graph-replayed training iterations: a TD7 pass between two step launches
    # under 2 ms apart (tools/iter_timeline.py); one from the bench's timed
    # window (the first run of them), past its warm-up
    pairs = [(a, b) for a, b in zip(starts[:-1], starts[1:])
             if any("encoder_kernel" in r["Kernel_Name"] for r in rows[a:b])
             and int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]) < 2_000_000]
    if not pairs:
        return None, []
    a, b = pairs[min(len(pairs) - 1, 100)]
    it = rows[a:b]
    wall = (int(rows[b]["Start_Timestamp"]) - int(it[0]["Start_Timestamp"])) / 1e3
    cls = {}
    for r in it:
        c = trace_iter.classify(r["Kernel_Name"])
        n, us = cls.get(c, (0, 0.0))
        cls[c] = (n + 1, us + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {"kernels": len(it), "wall_us": wall}, sorted(cls.items(), key=lambda x: -x[1][1])


def main():
    """usage: summarize.py ROUND TRAIN_DIR [ENV_DIR] [PMC_FETCH_DIR PMC_WRITE_DIR] [--bytes-per-launch B]"""
    args = sys.argv[1:]
    bpl = None
    if "--bytes-per-launch" in args:
        i = args.index("--bytes-per-launch")
        bpl = float(args[i + 1])
        del args[i:i + 2]
    rnd, stats = args[0], args[1]
    env_dir = args[2] if len(args) in (3, 5) else None
    pmc_dirs = args[-2:] if len(args) >= 4 else None
    here = os.path.dirname(os.path.abspath(__file__))
    ks = kernel_stats(stats)
    res = {"round": rnd, "kernels": ks[:40]}
    lines = [f"# rocprofv3 kernel summary ({rnd})", "", "Training bench (`bench.py`, default mode), all kernels:", "",
             "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for k in ks[:25]:
        lines.append(f"| `{k['name'][:90]}` | {k['calls']} | {k['total_ms']:.2f} | {k['avg_us']:.1f} | {k['pct']:.1f} |")
    meta, cls = iteration_classes(stats)
    if meta:
        res["iteration"] = dict(meta, classes={c: {"kernels": n, "us": us} for c, (n, us) in cls})
        lines += ["", f"One steady-state training iteration under the profiler: {meta['kernels']} kernels, "
                      f"{meta['wall_us']:.0f} us wall (tracing inflates short kernels):", "",
                  "| class | kernels | us |", "|---|---|---|"]
        lines += [f"| {c} | {n} | {us:.1f} |" for c, (n, us) in cls]
    if env_dir:
        ek = [k for k in kernel_stats(env_dir) if "exo_step" in k["name"]]
        res["env_mode_exo_step"] = ek
        lines += ["", "Env-only bench (`bench.py --mode env`), step kernel:", ""]
        lines += [f"- `{k['name'][:60]}`: {k['calls']} calls, avg {k['avg_us']:.2f} us" for k in ek]
    if pmc_dirs:
        f, w = pmc(pmc_dirs[0], "FETCH_SIZE"), pmc(pmc_dirs[1], "WRITE_SIZE")
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
