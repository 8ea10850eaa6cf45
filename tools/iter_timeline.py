"""Timeline of steady-state training iterations from a rocprofv3 kernel trace
(tools/trace_iter.sh): per iteration the wall span, the union of kernel busy
intervals, the idle gaps, and (with -v) every kernel's start offset, duration
and queue."""
import csv
import sys


def short(name):
    for p in ("void ", "td7dense::", "at::native::", "(anonymous namespace)::"):
        name = name.replace(p, "")
    return name.split("(")[0][:60]


def main(path, verbose=False):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows))
    steps = [i for i, k in enumerate(ks) if "exo_step" in k[2]]
    # training iterations (the bench's kernel-timing phase launches the step kernel alone)
    # (graph-replayed iterations: a TD7 pass between two step launches, under 2 ms)
    pairs = [(a, b) for a, b in zip(steps[:-1], steps[1:]) if b - a > 10
             and any("encoder_kernel" in k[2] for k in ks[a:b]) and ks[b][0] - ks[a][0] < 2_000_000][-6:-1]
    spans = []
    for a, b in pairs:
        it = ks[a:b]
        t0, t1 = it[0][0], ks[b][0]
        busy, cur_s, cur_e = 0, None, None
        for s, e, _, _ in it:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += min(cur_e, t1) - cur_s
        ksum = sum(e - s for s, e, _, _ in it)
        spans.append((t1 - t0, busy, ksum, len(it)))
        print(f"iteration: span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us,"
              f" sum of kernel durations {ksum / 1e3:.1f} us, {len(it)} kernels")
    if verbose:  # the last two iterations (one of each policy-update parity)
        for a, b in pairs[-2:]:
            t0 = ks[a][0]
            print(f"-- iteration of {(ks[b][0] - t0) / 1e3:.1f} us")
            for s, e, n, q in ks[a:b]:
                print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:>2}  {short(n)}")


if __name__ == "__main__":
    main(sys.argv[1], "-v" in sys.argv)
