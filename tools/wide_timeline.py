"""One steady-state iteration of the wide configuration (configs[4]) from a
rocprofv3 kernel trace: every kernel's start offset, duration and queue
between two consecutive env-step launches (exo_step_kernel), plus the
iteration span and busy time.  usage: wide_timeline.py kernel_trace.csv"""
import csv
import sys


def short(n):
    for p in ("void ", "td7dense::", "at::native::", "(anonymous namespace)::"):
        n = n.replace(p, "")
    return n.split("(")[0][:58]


rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
steps = [i for i, k in enumerate(ks) if "exo_step" in k[2]]
pairs = [(a, b) for a, b in zip(steps[:-1], steps[1:]) if b - a > 10 and ks[b][0] - ks[a][0] < 20_000_000]
for a, b in pairs[-2:]:
    t0, t1 = ks[a][0], ks[b][0]
    print(f"-- iteration span {(t1 - t0) / 1e3:.1f} us, {b - a} kernels")
    for s, e, n, q in ks[a:b]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>2}  {short(n)}")
