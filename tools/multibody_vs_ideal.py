"""Oracle study: the multibody stepSimulation (oracle/multibody.c) against the
idealised motor model on the reference's golden episodes
(tests/golden/env_m*.npz actions and draws).  Prints per motion the largest
joint-angle and observation differences, the solver's motor residual, the
number of limit rows and the largest prismatic displacement."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("oracle", "tests", "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"):
    sys.path.insert(0, os.path.join(REPO, p))
import oracle as O  # noqa: E402
from helpers import episode_steps, golden_env  # noqa: E402
from exo_amd import motions  # noqa: E402


def main(iters=50):
    angles, _ = motions.load()
    for m in range(8):
        d = golden_env(m)
        L = int(d["L"])
        envs = []
        for mode in ("ideal", "multibody"):
            e = O.OracleEnv(angles[m][:, :L], d["tremor_seq"], d["amp_range"], d["harm1"], d["harm2"],
                            d["max_force"][0], d["max_force"][1], d["dr"][0], d["dr"][1], d["dr"][2])
            e.set_physics(mode, O.mb_params(iters=iters))
            e.reset(d["ep0_draws"])
            envs.append(e)
        dq = dobs = res = pq = 0.0
        nlim = 0
        for ep in (1, 2):
            for e in envs:
                e.reset(d[f"ep{ep}_draws"])
            for k in episode_steps(d, ep):
                o1 = envs[0].step(d["step_action"][k])
                o2 = envs[1].step(d["step_action"][k])
                dq = max(dq, np.abs(envs[0].phys_q() - envs[1].phys_q()).max())
                dobs = max(dobs, np.abs(o1[0] - o2[0]).max())
                q, qd, st = envs[1].mb_state()
                res = max(res, st[1])
                nlim += int(st[0])
                pq = max(pq, np.abs(q[5:]).max())
        print(f"motion {m}: max|dq| {dq:.3e} rad  max|dobs| {dobs:.3e}  motor residual {res:.3e} rad/s  "
              f"limit rows {nlim}  max|q_prismatic| {pq:.3e} m")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
