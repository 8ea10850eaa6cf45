"""Kernel summary (calls, total ms, avg us, %) from a rocprofv3 rocpd SQLite
database (ROCm 7 default output).  usage: python tools/rocpd_summary.py DB [TOP]"""
import sqlite3
import sys


def summary(db, top=30):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select name, count(*), sum(end - start), avg(end - start) from kernels "
                       "group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = ["| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for name, n, s, a in rows[:top]:
        nm = name if len(name) <= 90 else name[:87] + "..."
        out.append(f"| `{nm}` | {n} | {s / 1e6:.2f} | {a / 1e3:.1f} | {100 * s / tot:.1f} |")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30))
