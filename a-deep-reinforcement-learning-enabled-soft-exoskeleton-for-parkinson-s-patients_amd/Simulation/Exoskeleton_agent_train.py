"""Training driver mirroring Simulation/Exoskeleton_agent_train.py of the
reference: the same command-line flags, the same per-step call sequence into
the drop-in env / agent, the same episode-round structure and checkpointing.

Call sequence kept (reference line numbers):
  construct one ExoskeletonEnv_train per reference motion (:60-71) and the
  Agent (:80-81); per episode round (:110): env.reset() +
  return_generated_tremor_data() for every env (:111-113); while any env runs
  (:123): per env select_action(obs) or a uniform random action before the
  warm-up ends (:125-131), env.step(action) (:141),
  replay_buffer.add(..., tremor_num=i) (:142), score / ep_len / step count and
  the tremor-suppression statistics (:144-200); after the round
  agent.maybe_train_and_checkpoint(round(mean(ep_len)), mean(score)) (:208),
  the warm-up switch (:210-211), the per-round metrics (:213-267) and
  agent.save (:290).

The reference script cannot run as shipped.  The fixes, each
marked "FIX n" below:
  FIX 1  :62-70   tremor_amplitude_range is a required constructor argument
                  the script never passes -> passed explicitly ([0.95, 1.05],
                  the range both evaluation scripts use; the drop-in env also
                  defaults to it).
  FIX 2  :128     select_action(obs) with a 1-D obs raised IndexError in
                  Actor.forward (TD7_multi_agent.py:74) -> the drop-in Agent
                  accepts (80,) and (N, 80) states; the call is unchanged.
  FIX 3  :128     select_action applied torch.randn_like / .clamp to a numpy
                  array (TD7_multi_agent.py:203-209) -> the drop-in Agent adds
                  Gaussian noise in numpy; the call is unchanged.
  FIX 4  :329     agent_rew[:, i] / std_score[:, i] index Python lists ->
                  converted to arrays first.
Other departures: stdout is not teed into a Logger and the reward curves are
saved as .npz instead of plotted (reporting layer, out of scope); --save_dir
replaces the hard-coded "AGENT_NNS/test_agent" prefix; --max_rounds bounds a
run for tests; --precision picks the TD7 MFMA operands (fp32 = the reference).
The vectorised form of this schedule is exo_amd.rollout.RefScheduleTrainer.
"""
import argparse
import os
import random
import sys
import time

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from Agent.TD7_multi_agent import Agent  # noqa: E402
from Environment.Exoskeleton_env import ExoskeletonEnv_train  # noqa: E402


def seed_everything(seed):
    """Utilities/seed_setting_.py:6-15."""
    import torch
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def dh_end_effector(theta, humerus, forearm, hand):
    """End-effector position of the 7-DOF Denavit-Hartenberg arm
    (Utilities/calculate_arm_end_effector_points.py:18-50); `hand` enters no
    transform there either."""
    alphas = (np.pi / 2, np.pi / 2, -np.pi / 2, np.pi / 2, np.pi / 2, np.pi / 2, np.pi / 2)
    ds = (0.0, 0.0, humerus, 0.0, forearm, 0.0, 0.0)
    T = np.eye(4)
    for al, d, th in zip(alphas, ds, theta):
        ct, st, ca, sa = np.cos(th), np.sin(th), np.cos(al), np.sin(al)
        T = T @ np.array([[ct, -st * ca, st * sa, 0.0], [st, ct * ca, -ct * sa, 0.0], [0.0, sa, ca, d],
                          [0.0, 0.0, 0.0, 1.0]])
    return T[:3, 3]


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--seed", default=0, type=int)
    p.add_argument("--n_steps", default=6e6, type=int)
    p.add_argument("--warmup", default=25e3, type=int)
    p.add_argument("--num_reference_motions", default=8, type=int)
    p.add_argument("--use_all_dof", default=False, action=argparse.BooleanOptionalAction)
    p.add_argument("--tremor_sequence", default=np.array([0, 1, 0, 1, 0, 0, 0]))
    p.add_argument("--first_harmonics_interval", default=np.array([4, 6]))
    p.add_argument("--second_harmonics_interval", default=np.array([8, 10]))
    p.add_argument("--dr_actuator_end_pos_shift", default=0.02, type=float)
    p.add_argument("--dr_actuator_range", default=0.03, type=float)
    p.add_argument("--dr_anatomical_matrix_noise", default=0.1, type=float)
    p.add_argument("--humerus_length", default=0.4, type=float)
    p.add_argument("--humerus_radius", default=0.05, type=float)
    p.add_argument("--forearm_length", default=0.4, type=float)
    p.add_argument("--forearm_radius", default=0.05, type=float)
    p.add_argument("--hand_length", default=0.05, type=float)
    p.add_argument("--max_force_elbow", default=20, type=float)
    p.add_argument("--max_force_shoulder", default=40, type=float)
    p.add_argument("--print_each_env_data", default=False, action=argparse.BooleanOptionalAction)
    p.add_argument("--print_tremor_data", default=False, action=argparse.BooleanOptionalAction)
    # mirror-only
    p.add_argument("--save_dir", default="AGENT_NNS", help="checkpoint directory (reference: AGENT_NNS)")
    p.add_argument("--max_rounds", default=None, type=int, help="stop after this many episode rounds")
    p.add_argument("--buffer_size", default=None, type=int, help="LAP rows per env (reference: 2.5e5)")
    p.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "fp16"],
                   help="TD7 MFMA operands (reference: fp32)")
    p.add_argument("--quiet", default=False, action="store_true")
    return p.parse_args(argv)


class StepStats:
    """Per-step tremor-suppression statistics of one episode round
    (Simulation/Exoskeleton_agent_train.py:116-121, 133-205)."""

    def __init__(self, n_envs, disregard=True):
        self.n = n_envs
        self.disregard = disregard
        self.torque_red, self.ampl_red, self.ampl_total_red = [], [], []
        self.when_red = np.zeros((n_envs, 2))       # [>= 0, < 0] counts over axes 0-3
        self.when_ampl_red = np.zeros((n_envs, 2))  # [>= 0, < 0] counts of the total amplitude change
        self.red_in_episode = np.zeros(n_envs)

    def begin_step(self):
        self._t = np.zeros((self.n, 7))
        self._a = np.zeros((self.n, 7))
        self._tot = np.zeros(self.n)

    def record(self, i, info, base_deg, args):
        with np.errstate(divide="ignore", invalid="ignore"):
            tr = (np.abs(info["torque_val"]) - np.abs(info["tremor_torque_val"])) / np.abs(info["tremor_torque_val"])
            ar = (np.abs(info["ampl_val"]) - np.abs(info["tremor_ampl_val"])) / np.abs(info["tremor_ampl_val"])
        tr = np.nan_to_num(tr * 100, nan=0, posinf=0, neginf=0)
        ar = np.nan_to_num(ar * 100, nan=0, posinf=0, neginf=0)
        base = np.radians(base_deg)
        geo = (args.humerus_length, args.forearm_length, args.hand_length)
        p0 = dh_end_effector(base, *geo)
        d_sup = np.linalg.norm(dh_end_effector(np.radians(info["ampl_val"]) + base, *geo) - p0)
        d_uns = np.linalg.norm(dh_end_effector(np.radians(info["tremor_ampl_val"]) + base, *geo) - p0)
        total = (d_sup - d_uns) / d_uns * 100
        self.when_red[i] += [np.sum(tr[:4] >= 0), np.sum(tr[:4] < 0)]
        self.red_in_episode[i] += bool(np.any(tr[:4] < 0))
        if total < 0:
            self.when_ampl_red[i, 1] += 1
            self._tot[i] = total
        else:
            self.when_ampl_red[i, 0] += 1
        if self.disregard:  # keep suppression only
            tr[tr > 0] = 0
            ar[ar > 0] = 0
        if np.count_nonzero(tr):
            self._t[i] = tr
        if np.count_nonzero(ar):
            self._a[i] = ar

    def end_step(self):
        self.torque_red.append(self._t)
        self.ampl_red.append(self._a)
        self.ampl_total_red.append(self._tot)


def train(args):
    t_start = time.time()
    seed_everything(args.seed)
    envs = [ExoskeletonEnv_train(reference_motion_file_num=str(m),
                                 tremor_sequence=args.tremor_sequence,
                                 tremor_amplitude_range=np.array([0.95, 1.05]),  # FIX 1 (:62-70)
                                 first_harmonics_interval=args.first_harmonics_interval,
                                 second_harmonics_interval=args.second_harmonics_interval,
                                 max_force_shoulder=args.max_force_shoulder,
                                 max_force_elbow=args.max_force_elbow,
                                 dr_actuator_end_pos_shift=args.dr_actuator_end_pos_shift,
                                 dr_actuator_range=args.dr_actuator_range,
                                 matrix_noise_fraction=args.dr_anatomical_matrix_noise)
            for m in range(args.num_reference_motions)]
    E = len(envs)
    obs_dim, act_dim = envs[0].observation_space.shape[0], envs[0].action_space.shape[0]
    agent = Agent(state_dim=obs_dim, action_dim=act_dim, max_action=1, learning_steps=args.n_steps, env_num=E,
                  buffer_size=args.buffer_size, precision=args.precision)
    max_lengths = [env.return_max_length() for env in envs]
    steps_per_round = sum(max_lengths)
    os.makedirs(args.save_dir, exist_ok=True)
    save_prefix = os.path.join(args.save_dir, "test_agent")
    initial_score, disregard = 2, True
    allow_train = False
    steps_count, rounds = 0, 0
    scores, agent_rew, avg_agent_rew, std_score, median_tremor_sup = [], [], [], [], []
    round_stats = []  # the global outputs of every round (:292-317), for comparisons
    sup_avg_hist = []
    observation = np.zeros((E, obs_dim))
    actions = np.zeros((E, act_dim))
    score = np.zeros(E)
    torque_places, torque_maxes = np.zeros((E, 7)), np.zeros((E, 7))
    log = (lambda *a: None) if args.quiet else print

    while steps_count < args.n_steps and (args.max_rounds is None or rounds < args.max_rounds):
        for i, env in enumerate(envs):
            observation[i], score[i] = env.reset()
            torque_places[i], torque_maxes[i] = env.return_generated_tremor_data()
        done = np.zeros(E, dtype=bool)
        ep_len = np.ones(E, dtype=int)
        stats = StepStats(E, disregard)
        while not done.all():
            for i in np.flatnonzero(~done):
                if allow_train:
                    actions[i] = agent.select_action(observation[i], use_checkpoint=False,  # FIX 2, FIX 3
                                                     use_exploration=True)
                else:
                    actions[i] = np.clip(np.random.uniform(-1, 1, act_dim), -1, 1)
            stats.begin_step()
            for i in np.flatnonzero(~done):
                nxt, reward, done[i], _, info = envs[i].step(actions[i])
                agent.replay_buffer.add(observation[i], actions[i], nxt, reward, done[i], tremor_num=i)
                score[i] += reward
                ep_len[i] += 1
                steps_count += 1
                observation[i] = nxt
                stats.record(i, info, envs[i].return_original_joint_angles(), args)
            stats.end_step()

        agent.maybe_train_and_checkpoint(ep_timesteps=round(np.mean(ep_len)), ep_return=np.mean(score))
        if steps_count > args.warmup:
            allow_train = True
        rounds += 1

        # per-round metrics (:213-267)
        gotten = score - initial_score
        pct = gotten / ep_len * 100
        scores.append(score.copy())
        agent_rew.append(pct)
        avg_r = np.mean(agent_rew[-100:], axis=0)
        avg_agent_rew.append(avg_r)
        tred = np.array(stats.torque_red)     # [steps, E, 7]
        ared = np.array(stats.ampl_red)
        tot = np.array(stats.ampl_total_red)  # [steps, E]
        sup_avg, sup_med = np.zeros(E), np.zeros(E)
        for i in range(E):
            t_i = tred[:max_lengths[i], i]
            nz = t_i[t_i != 0]
            sup_avg[i] = nz.mean() if nz.size else np.nan
            sup_med[i] = np.median(nz) if nz.size else np.nan
            sup_avg_hist.append(t_i.mean(axis=0))
            if args.print_each_env_data:
                log(f"\nReference movement {i}: score {score[i]:.3f}, reward % {pct[i]:.3f}, "
                    f"tremor suppression avg {sup_avg[i]:.3f}% median {sup_med[i]:.3f}%, "
                    f"amplitude suppression {tot[:max_lengths[i], i].mean():.3f}%, "
                    f"torque places {torque_places[i]}, max Nm {torque_maxes[i]}")
        agent.save(save_prefix)
        with np.errstate(invalid="ignore"):
            occ = np.sum(stats.when_red[:, 1]) / np.sum(stats.when_red) * 100
            occ_a = np.sum(stats.when_ampl_red[:, 1]) / np.sum(stats.when_ampl_red) * 100
            nz_tot = tot[tot != 0]
            nz_a = ared[ared != 0]
        log(f"\nGLOBAL TRAINING OUTPUTS (round {rounds}): steps {steps_count}, "
            f"avg reward {np.mean(gotten):.3f}, reward % {np.mean(pct):.3f}, avg rewards % {np.mean(avg_r):.3f}, "
            f"median {np.median(avg_r):.3f}; tremor reduction in {occ:.2f}% of axis-steps, any-axis reduction in "
            f"{np.sum(stats.red_in_episode) / steps_per_round * 100:.2f}% of the episode, overall suppression "
            f"avg {np.nanmean(sup_avg):.3f}% median {np.nanmean(sup_med):.3f}%; angle suppression "
            f"{(nz_a.mean() if nz_a.size else 0.0):.3f}%, amplitude reduction in {occ_a:.2f}% of steps, "
            f"total amplitude suppression {(nz_tot.mean() if nz_tot.size else 0.0):.3f}%")
        round_stats.append(dict(
            avg_reward=float(np.mean(gotten)), reward_pct=float(np.mean(pct)), avg_rewards_pct=float(np.mean(avg_r)),
            median_rewards_pct=float(np.median(avg_r)), tremor_reduction_occurrence=float(occ),
            any_axis_reduction_pct=float(np.sum(stats.red_in_episode) / steps_per_round * 100),
            overall_suppression_avg=float(np.nanmean(sup_avg)), overall_suppression_median=float(np.nanmean(sup_med)),
            angle_suppression=float(nz_a.mean() if nz_a.size else 0.0), amplitude_reduction_occurrence=float(occ_a),
            total_amplitude_suppression=float(nz_tot.mean() if nz_tot.size else 0.0),
            suppression_avg_per_env=sup_avg.copy(), suppression_median_per_env=sup_med.copy()))
        std_score.append(np.std(avg_agent_rew[-100:], axis=0))
        median_tremor_sup.append(np.nanmean(sup_med))

    for env in envs:
        env.close()
    # FIX 4 (:329): the curves are lists of per-round arrays
    agent_rew_a, std_a = np.array(agent_rew), np.array(std_score)
    np.savez(os.path.join(args.save_dir, "algo_score.npz"), score=agent_rew_a, std=std_a)
    h, rem = divmod(int(time.time() - t_start), 3600)
    log(f"Script executed in {h} hours, {rem // 60} minutes, and {rem % 60} seconds.")
    return dict(agent=agent, steps=steps_count, rounds=rounds, scores=np.array(scores), agent_rew=agent_rew_a,
                save_prefix=save_prefix, round_stats=round_stats)


if __name__ == "__main__":
    train(parse_args())
