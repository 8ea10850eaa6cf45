"""Reference motions (IMU joint angles at 40 Hz).

data/motions.npz holds the 5 angle columns of
Simulation/reference_motions/ref_motion_{0..7}.txt as parsed by
Utilities/read_txt_env.py:109-113 (columns elbow_y, elbow_z, shoulder_x,
shoulder_y, shoulder_z, in degrees), padded to the longest motion.
"""
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "motions.npz")
_cache = None


def load():
    """Returns (angles_deg [n_motions, 5, max_len] float64, lengths [n_motions] int32)."""
    global _cache
    if _cache is None:
        d = np.load(_PATH, allow_pickle=False)
        _cache = (np.ascontiguousarray(d["angles_deg"], dtype=np.float64),
                  np.ascontiguousarray(d["lengths"], dtype=np.int32))
    return _cache


def n_motions():
    return load()[1].size
