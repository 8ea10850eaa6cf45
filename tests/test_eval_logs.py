"""The authors' evaluation logs (tests/golden/eval_log_stats.json, extracted by
tools/parse_eval_logs.py from /root/reference/Evaluation_logs): the facts
profiles/r03_eval_hypotheses.md builds on.  CPU, data only."""
import json

import numpy as np

from helpers import GOLDEN

# the maxima of Utilities/generate_parkinson_tremor.py:44's docstring order
# (shoulder z 10, y 5, x 2.5, elbow 5); the shipped :59 has [2.5, 5, 10, 5]
LOG_MAXIMA = np.array([10.0, 5.0, 2.5, 5.0, 0.0, 0.0, 0.0])


def _stats():
    return json.load(open(f"{GOLDEN}/eval_log_stats.json"))


def test_logs_print_unit_magnitude_docstring_maxima():
    """Every per-env block of every configuration prints the episode's max
    tremor torque as exactly the docstring-order maxima on its tremor axes
    (std 0 over the 100 episodes): no magnitude draw in [0.95, 1.05], no
    per-sample sign flip, axes 0 and 2 swapped against the shipped table."""
    st = _stats()
    assert len(st) == 15
    for cfg, per in st.items():
        seq = np.array([int(c) for c in cfg.strip("[]").split(",")] + [0, 0, 0])
        for m in range(8):
            d = per[str(m)]
            assert d["episodes"] == 100
            np.testing.assert_array_equal(d["max_nm"]["mean"], LOG_MAXIMA * seq, err_msg=f"{cfg} motion {m}")
            np.testing.assert_array_equal(d["max_nm"]["std"], np.zeros(7), err_msg=f"{cfg} motion {m}")


def test_log_statistics_are_consistent_with_the_evaluation_metrics():
    """The per-env 'Total tremor amplitude suppression' lines average to the
    sign of the log's EVALUATION METRICS (every configuration reduces the
    amplitude on average) and the occurrences are percentages."""
    for cfg, per in _stats().items():
        tot = np.mean([per[str(m)]["ampl_total"]["mean"] for m in range(8)])
        assert tot < 0, cfg
        for m in range(8):
            for k in ("torque_all", "torque_any", "ampl_occurrence"):
                assert 0 <= per[str(m)][k]["mean"] <= 100, (cfg, m, k)
