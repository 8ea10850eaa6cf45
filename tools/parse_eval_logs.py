"""Per-motion statistics of the authors' evaluation logs
(/root/reference/Evaluation_logs/<cfg>: stdout of Simulation/Evaluate_control_
performance.py, 100 episodes x 8 envs, seed 0).  Every episode prints one
"TREMOR i statistics" block per env (:310-337); this collects, per
configuration and motion i, the mean / std over the 100 episodes of

  score            episode return incl. the reset's 2 (:313)
  pct_to_max       (score - 2) / ep_len * 100 (:274-275, :315)
  torque_all       steps with every tremor axis' torque suppressed / (L - 3) * 100 (:230, :321)
  torque_any       steps with some tremor axis suppressed / (L - 3) * 100 (:232, :325-327)
  ampl_occurrence  steps with the total amplitude reduced / L * 100 (:235-236, :332)
  ampl_total       mean over the first L entries of the per-step total amplitude change,
                   positive changes zeroed (:219, :245-246, :336)
  ampl_axis[7]     mean per-axis angle-amplitude change, positive changes zeroed (:192-193, :244, :329)
  max_nm[7]        printed max of the episode's tremor table (:337, return_generated_tremor_data)

and writes them (numbers only) to tests/golden/eval_log_stats.json.

usage: python tools/parse_eval_logs.py [--logs /root/reference/Evaluation_logs]
"""
import argparse
import json
import os
import re

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NUM = r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?|nan"


def _vec(s):
    return [float(v) for v in re.findall(NUM, s)]


def parse(path):
    text = open(path).read()
    blocks = re.split(r"\nTREMOR (\d) statistics: ?\n", "\n" + text)
    out = {m: {k: [] for k in ("score", "pct_to_max", "torque_all", "torque_any", "ampl_occurrence",
                               "ampl_total", "ampl_axis", "max_nm")} for m in range(8)}
    for k in range(1, len(blocks) - 1, 2):
        m, b = int(blocks[k]), blocks[k + 1]
        b = b.split("GLOBAL TRAINING OUTPUTS")[0]
        g = lambda pat: re.search(pat, b).group(1)  # noqa: E731
        d = out[m]
        d["score"].append(float(g(r"^ score (" + NUM + ")")))
        d["pct_to_max"].append(float(g(r"Score in percent to max: (" + NUM + ")")))
        d["torque_all"].append(float(g(r"Tremor reduction occurred in (" + NUM + ") % of all the generated")))
        d["torque_any"].append(float(g(r"along any axis in (" + NUM + ") % of the episode")))
        d["ampl_occurrence"].append(float(g(r"Tremor amplitude reduction occurred in (" + NUM + ") % of all time")))
        d["ampl_total"].append(float(g(r"Total tremor amplitude suppression (" + NUM + ") %")))
        amp = b.split("Tremor amplitude reduction metrics:")[1]
        d["ampl_axis"].append(_vec(re.search(r"Tremor reduction ep avg \[([^\]]*)\]", amp).group(1)))
        d["max_nm"].append(_vec(re.search(r"With maximum Nm of: \[([^\]]*)\]", b).group(1)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--logs", default="/root/reference/Evaluation_logs")
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "eval_log_stats.json"))
    a = ap.parse_args()
    res = {}
    for cfg in sorted(os.listdir(a.logs)):
        per = parse(os.path.join(a.logs, cfg))
        res[cfg] = {}
        for m in range(8):
            d = per[m]
            n = len(d["score"])
            assert n == 100, (cfg, m, n)
            res[cfg][str(m)] = {k: {"mean": np.mean(np.array(v, dtype=float), axis=0).round(6).tolist(),
                                    "std": np.std(np.array(v, dtype=float), axis=0).round(6).tolist()}
                                for k, v in d.items()}
            res[cfg][str(m)]["episodes"] = n
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=0)
    print("wrote", a.out)
    for cfg, r in res.items():
        print(cfg, " ".join(f"{r[str(m)]['ampl_total']['mean']:7.2f}" for m in range(8)),
              "| score", " ".join(f"{r[str(m)]['score']['mean']:6.1f}" for m in range(8)))


if __name__ == "__main__":
    main()
