"""Oracle (test infrastructure only) for the tremor-suppression statistics of
Simulation/Exoskeleton_agent_train.py:149-200 and the Denavit-Hartenberg arm
forward kinematics of Utilities/calculate_arm_end_effector_points.py:18-50 --
a numpy restatement, pinned by tests/golden/dh_fk.npz and
tests/golden/metrics_cases.npz (generated from the reference by
tests/golden/make_metrics_golden.py)."""
import numpy as np


def dh_matrix(alpha, a, d, theta):
    """calculate_arm_end_effector_points.py:8-15"""
    ct, st, ca, sa = np.cos(theta), np.sin(theta), np.cos(alpha), np.sin(alpha)
    return np.array([[ct, -st * ca, st * sa, a * ct], [st, ct * ca, -ct * sa, a * st], [0, sa, ca, d],
                     [0, 0, 0, 1]])


def end_effector(theta, L1, L2, L3):
    """calculate_arm_end_effector_points.py:18-50 (L3 is unused by the DH table)."""
    table = [(np.pi / 2, 0, 0), (np.pi / 2, 0, 0), (-np.pi / 2, 0, L1), (np.pi / 2, 0, 0), (np.pi / 2, 0, L2),
             (np.pi / 2, 0, 0), (np.pi / 2, 0, 0)]
    T = np.eye(4)
    for (alpha, a, d), th in zip(table, theta):
        T = T @ dh_matrix(alpha, a, d, th)
    return T[:3, 3]


def step_metrics(torque_val, tremor_torque_val, ampl_val, tremor_ampl_val, original_deg, lengths=(0.4, 0.4, 0.05),
                 disregard=True):
    """One env-step of Exoskeleton_agent_train.py:149-191: returns
    (tremor_reduction[7], tremor_reduction_ampl[7], ampl_total, counter deltas[5], last_negative_total or None)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        tr = np.nan_to_num((np.abs(torque_val) - np.abs(tremor_torque_val)) / np.abs(tremor_torque_val) * 100,
                           nan=0, posinf=0, neginf=0)
        ta = np.nan_to_num((np.abs(ampl_val) - np.abs(tremor_ampl_val)) / np.abs(tremor_ampl_val) * 100,
                           nan=0, posinf=0, neginf=0)
    orig = np.radians(np.asarray(original_deg, dtype=np.float64))
    p0 = end_effector(orig, *lengths)
    p1 = end_effector(np.radians(ampl_val) + orig, *lengths)
    p2 = end_effector(np.radians(tremor_ampl_val) + orig, *lengths)
    ds, du = np.linalg.norm(p1 - p0), np.linalg.norm(p2 - p0)
    total = (ds - du) / du * 100
    deltas = np.array([np.sum(tr[:4] >= 0), np.sum(tr[:4] < 0), float(np.any(tr[:4] < 0)),
                       float(not total < 0), float(total < 0)])
    last_neg = total if total < 0 else None
    if disregard:
        tr = np.where(tr > 0, 0, tr)
        ta = np.where(ta > 0, 0, ta)
        total = 0 if total > 0 else total
    return tr, ta, total, deltas, last_neg


def eval_step_counters(torque_val, tremor_torque_val, ampl_val, tremor_ampl_val, original_deg, tremor_sequence,
                       lengths=(0.4, 0.4, 0.05)):
    """One env-step of Simulation/Evaluate_control_performance.py:192-247: the
    counter deltas [all tremor axes suppressed, any tremor axis suppressed,
    total < 0, total >= 0, total if < 0 else 0] (exo_eval_metrics's counters)."""
    eps = 1e-10
    with np.errstate(divide="ignore", invalid="ignore"):
        tr = np.nan_to_num((np.abs(torque_val) - np.abs(tremor_torque_val)) / np.abs(tremor_torque_val + eps) * 100,
                           nan=0, posinf=0, neginf=0)
    sel = tr[np.asarray(tremor_sequence)[:7] == 1]
    orig = np.radians(np.asarray(original_deg, dtype=np.float64))
    a = np.array(ampl_val, dtype=np.float64)
    u = np.array(tremor_ampl_val, dtype=np.float64)
    a[[0, 1]] = a[[1, 0]]  # :208-209
    u[[0, 1]] = u[[1, 0]]
    p0 = end_effector(orig, *lengths)
    p1 = end_effector(np.radians(a) + orig, *lengths)
    p2 = end_effector(np.radians(u) + orig, *lengths)
    ds, du = np.linalg.norm(p1 - p0), np.linalg.norm(p2 - p0)
    total = (ds - du) / du * 100
    return np.array([float(np.all(sel <= 0)), float(np.any(sel <= 0)), float(total < 0), float(not total < 0),
                     total if total < 0 else 0.0])
