"""Drop-in ``ExoskeletonEnv_train`` (reference: Environment/Exoskeleton_env.py:34).

Same constructor arguments, attributes and methods as the reference gym env;
each instance is a one-env view of :class:`exo_amd.VecExoskeletonEnv`, whose
step/reset run as HIP kernels on the GPU.  Differences, all deliberate:

* ``tremor_amplitude_range`` defaults to [0.95, 1.05] (the reference requires
  it but its training script never passes it: Exoskeleton_agent_train.py:62-70).
* Randomness comes from Philox streams keyed by a seed drawn from the global
  ``np.random`` state at construction (so ``set_seeds`` keeps runs repeatable);
  the reference draws from ``np.random`` directly.
* PyBullet is replaced by URDF forward kinematics plus the idealised position
  motor model of SURVEY.md A.2 (default), or with ``physics="multibody"`` by
  Featherstone dynamics of the URDF tree with a joint-space impulse solve of
  the motors and limits (Bullet parity is unpinned).
* ``check_movement_boundaries`` counts violations instead of printing them.
"""
import numpy as np
import torch

from exo_amd.vec_env import DEFAULTS, VecExoskeletonEnv


class Box:
    """Minimal stand-in for gym.spaces.Box (gym is not a dependency)."""

    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is None:
            shape = np.asarray(low).shape
        self.shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), self.shape)
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), self.shape)
        self.dtype = np.dtype(dtype)

    def sample(self):
        return np.random.uniform(self.low, self.high).astype(self.dtype)


class ExoskeletonEnv_train:
    metadata = {'render.modes': ['human']}

    def __init__(self, reference_motion_file_num: str, tremor_sequence, tremor_amplitude_range=(0.95, 1.05),
                 first_harmonics_interval=(4, 6), second_harmonics_interval=(8, 10), max_force_shoulder: float = 40,
                 max_force_elbow: float = 20, dr_actuator_end_pos_shift: float = 0.02, dr_actuator_range: float = 0.1,
                 matrix_noise_fraction: float = 0.1, seed=None, device=None, physics="ideal"):
        self.file_num = str(reference_motion_file_num)
        self.dt = 1 / 40
        self.tremor_input_sequence = np.asarray(tremor_sequence)
        self.tremor_amplitude_range = np.asarray(tremor_amplitude_range, dtype=np.float64)
        self.tremor_axis_n = int(np.sum(self.tremor_input_sequence))
        self.first_harmonics_interval = np.asarray(first_harmonics_interval, dtype=np.float64)
        self.second_harmonics_interval = np.asarray(second_harmonics_interval, dtype=np.float64)
        self.max_output_shoulder_original = float(max_force_shoulder)
        self.max_output_elbow_original = float(max_force_elbow)
        self.dummy_shift_max_range = float(dr_actuator_end_pos_shift)
        self.actuator_domain_randomization_range = float(dr_actuator_range)
        self.matrix_noise_fraction = float(matrix_noise_fraction)
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 62))
        self._vec = VecExoskeletonEnv(1, motions=[int(self.file_num)], seed=seed, device=device,
                                      tremor_sequence=self.tremor_input_sequence,
                                      tremor_amplitude_range=self.tremor_amplitude_range,
                                      first_harmonics_interval=self.first_harmonics_interval,
                                      second_harmonics_interval=self.second_harmonics_interval,
                                      max_force_shoulder=max_force_shoulder, max_force_elbow=max_force_elbow,
                                      dr_actuator_end_pos_shift=dr_actuator_end_pos_shift,
                                      dr_actuator_range=dr_actuator_range,
                                      matrix_noise_fraction=matrix_noise_fraction, physics=physics)
        self.device = self._vec.device
        self.max_count = int(self._vec.lengths_host[0])
        self.action_space = Box(-1.0, 1.0, shape=(7,), dtype=np.float32)  # :74
        low = np.concatenate([np.repeat(0.0, 14), np.repeat(-15.0, 12), np.repeat(-2.0, 54)]).astype(np.float32)
        high = np.concatenate([np.repeat(1.5, 14), np.repeat(15.0, 12), np.repeat(2.0, 54)]).astype(np.float32)
        self.observation_space = Box(low, high, dtype=np.float32)  # :99-111 (not enforced)
        self.max_reward = float(self._vec.max_reward[0])  # :167-169
        self.epsilon = 1e-10
        self._done = False
        self._out = self._vec.new_outputs(True)
        # the constructor runs initialize_movement() (:172); exo_create did it on the device
        self.state = self._vec.reset()[0].cpu().numpy()

    # gym API ------------------------------------------------------------
    def reset(self):
        self.state = self._vec.reset()[0].cpu().numpy()
        self._done = False
        return self.state, self.counts  # (obs, 2): :473-478

    def step(self, action):
        if self._done:
            # the reference indexes past its episode buffers here (IndexError at :502-513)
            raise IndexError("step() called after the episode ended; call reset()")
        a = torch.as_tensor(np.asarray(action, dtype=np.float32).reshape(1, 7), device=self.device)
        obs, rew, done, info = self._vec.step(a, out=self._out)
        obs_h, rew_h, done_h, info_h = obs.cpu().numpy()[0], float(rew.cpu()[0]), bool(done.cpu()[0]), \
            info.cpu().numpy()[0]
        self._done = done_h
        info_d = VecExoskeletonEnv.unpack_info(info_h)
        self.state = obs_h
        return obs_h, rew_h, done_h, False, info_d

    def seed(self, seed=None):
        seed = int(np.random.randint(0, 2 ** 62)) if seed is None else int(seed)
        from exo_amd import _native as nat
        nat.check(nat.lib().exo_set_seed(self._vec._ctx, seed), "exo_set_seed")
        return [seed]

    def render(self, mode="human"):
        raise NotImplementedError("no GUI: the simulation runs as HIP kernels")

    def close(self):
        self._vec.close()

    # accessors (:572-592) -------------------------------------------------
    @property
    def counts(self):
        return int(self._vec.get_state(0)[0])

    @property
    def max_output_shoulder(self):
        return float(self._vec.get_state(0)[47])

    @property
    def max_output_elbow(self):
        return float(self._vec.get_state(0)[48])

    @property
    def tremor_torque_values(self):
        return self._vec.tremor(0)

    def return_generated_tremor_data(self):
        return self.tremor_input_sequence, self.tremor_torque_values.max(axis=1)

    def return_max_length(self) -> int:
        return self.max_count

    def return_original_joint_angles(self) -> list:
        return list(self._vec.original_joint_angles(0))

    @property
    def boundary_violations(self):
        """Steps whose commanded angles left the ranges of check_movement_boundaries (:594-605)."""
        return int(self._vec.get_state(0)[52])

    def check_movement_boundaries(self):
        return self.boundary_violations


__all__ = ["ExoskeletonEnv_train", "DEFAULTS"]
