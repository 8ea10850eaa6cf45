"""Golden vectors for the tremor-suppression statistics (run here, where the
reference is importable; the output travels, the reference does not):
  dh_fk.npz        -- Utilities/calculate_arm_end_effector_points.forward_kinematics
                      on random joint angles and arm lengths;
  metrics_cases.npz -- the per-step formulas of Simulation/Exoskeleton_agent_train.py:149-191
                      evaluated with the reference's forward_kinematics / distance_3d.
usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_metrics_golden.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")
from Utilities.calculate_arm_end_effector_points import distance_3d, forward_kinematics  # noqa: E402


def main():
    rng = np.random.default_rng(7)
    th = rng.uniform(-1.6, 1.6, size=(64, 7))
    lens = rng.uniform(0.2, 0.5, size=(64, 3))
    pos = np.stack([forward_kinematics(t, *l) for t, l in zip(th, lens)])
    np.savez(os.path.join(HERE, "dh_fk.npz"), theta=th, lengths=lens, position=pos)

    n = 48
    tq = rng.normal(size=(n, 7)) * 2
    ttq = rng.normal(size=(n, 7)) * 2
    ttq[::7, 5] = 0.0                       # zero tremor torque -> nan_to_num path
    am = rng.normal(size=(n, 7)) * 3
    tam = rng.normal(size=(n, 7)) * 3
    tam[::5, 6] = 0.0
    orig = np.concatenate([rng.uniform(-60, 60, size=(n, 5)), np.zeros((n, 2))], 1)
    L1, L2, L3 = 0.4, 0.4, 0.05
    tr_o, ta_o, tot_o, cnt_o = [], [], [], []
    for k in range(n):
        with np.errstate(divide="ignore", invalid="ignore"):
            tr = np.nan_to_num((abs(tq[k]) - abs(ttq[k])) / abs(ttq[k]) * 100, nan=0, posinf=0, neginf=0)
            ta = np.nan_to_num((abs(am[k]) - abs(tam[k])) / abs(tam[k]) * 100, nan=0, posinf=0, neginf=0)
        non = np.radians(orig[k])
        e0 = forward_kinematics(non, L1, L2, L3)
        e1 = forward_kinematics(np.radians(am[k]) + non, L1, L2, L3)
        e2 = forward_kinematics(np.radians(tam[k]) + non, L1, L2, L3)
        ds, du = distance_3d(e0, e1), distance_3d(e0, e2)
        tot = ((ds - du) / du) * 100
        cnt = [np.sum(tr[:4] >= 0), np.sum(tr[:4] < 0), float(np.any(tr[:4] < 0)), float(not tot < 0), float(tot < 0)]
        tr[tr > 0] = 0
        ta[ta > 0] = 0
        if tot > 0:
            tot = 0
        tr_o.append(tr), ta_o.append(ta), tot_o.append(tot), cnt_o.append(cnt)
    np.savez(os.path.join(HERE, "metrics_cases.npz"), torque_val=tq, tremor_torque_val=ttq, ampl_val=am,
             tremor_ampl_val=tam, original_deg=orig, tremor_reduction=np.array(tr_o),
             tremor_reduction_ampl=np.array(ta_o), ampl_total=np.array(tot_o), counter_deltas=np.array(cnt_o))
    print("wrote dh_fk.npz, metrics_cases.npz")


if __name__ == "__main__":
    main()
