"""Per-tensor report of tests/test_td7_full.py: for every gradient, the
distance from the reference golden, from the teacher-forced fp64 restatement
(same operand rounding) and the golden's own distance from exact arithmetic
("noise").  usage: python tools/diag_td7_full.py golden precision"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import conftest  # noqa: E402,F401
import test_td7_full as t  # noqa: E402

golden, prec = sys.argv[1], sys.argv[2]
orig = t._check_grads


def check(g, step, L, mnames, precision, report, free, forced):
    for mname in mnames:
        for name, tt in t._named(getattr(L, mname), mname, grad=True).items():
            key = f"step{step}_grad.{name}"
            xs, _ = t._sample(name, tt)
            print(f"{golden} {prec} step {step} {name:24s} golden {t._rel(xs, g[key]):.2e}  forced "
                  f"{t._rel(xs, forced[key]):.2e}  noise {free['noise'][key]:.2e}  forced-vs-golden "
                  f"{t._rel(forced[key], g[key]):.2e}", flush=True)
    return 0.0


t._check_grads = check
try:
    t._run("cuda", prec, golden=golden)
except AssertionError as e:
    print("assert:", str(e)[:300])
