"""Pink-noise exploration and select_action (T5) against the
reference.

tests/golden/pink.npz (make_golden.py --only pink) holds
* Agent/colorednoise.powerlaw_psd_gaussian (:9-124) outputs for seeded
  np.random.Generators (several exponents, shapes, a low-frequency cut-off);
* two episodes of the Pink agent's exploring select_action
  (Agent/TD7_multi_agent_Pink_noise.py:203-228) with the episode noise
  generators seeded (77, 78): the noise buffers, the actions of every call and
  hp.exploration_noise after it (one decrement per call, :225).

tests/golden/select_action.npz holds the batched select_action with
exploration off, checkpoint and live nets.

Tolerances: the numpy coloured noise is the same float64 arithmetic (1e-12);
actions go through fp32 nets (1e-5 on the GPU's f32 MFMA); the device noise is
float32 after a float64 irfft (1e-6)."""
import numpy as np
import pytest
import torch

from helpers import GOLDEN

PINK_CASES = [(1.0, (7, 344), 0.0, 11), (1.0, (7, 229), 0.0, 12), (1.0, (7, 341), 0.0, 13), (2.0, (3, 100), 0.0, 14),
              (0.5, (7, 64), 0.0, 15), (1.0, (2, 50), 0.1, 16), (1.0, 33, 0.0, 17)]  # = make_golden.PINK_CASES


def _g():
    return np.load(f"{GOLDEN}/pink.npz", allow_pickle=False)


def _sd(g, prefix):
    return {k[len(prefix) + 1:]: torch.tensor(g[k]) for k in g.files if k.startswith(prefix + ".")}


def test_powerlaw_noise_matches_reference_generator():
    from exo_amd.pink import powerlaw_psd_gaussian
    g = _g()
    for k, (beta, size, fmin, seed) in enumerate(PINK_CASES):
        x = powerlaw_psd_gaussian(beta, size, fmin=fmin, rng=np.random.default_rng(seed))
        np.testing.assert_allclose(x, g[f"case{k}"], rtol=1e-12, atol=1e-12, err_msg=f"case {k}")


def _spectrum(seed, rows, n, beta=1.0):
    """The scaled Gaussian spectra a seeded Generator gives colorednoise.py:104-105."""
    from exo_amd.pink import _spectrum_scale
    scale, _ = _spectrum_scale(beta, n)
    rng = np.random.default_rng(seed)
    sr = rng.normal(scale=scale, size=(rows, scale.size))
    si = rng.normal(scale=scale, size=(rows, scale.size))
    return sr, si


def _agent(g):
    from exo_amd.td7 import Agent, Hyperparameters
    hp = Hyperparameters(zs_dim=16, enc_hdim=24, critic_hdim=20, actor_hdim=18)
    ag = Agent(80, 7, 1, learning_steps=int(g["learning_steps"]), hp=hp, env_num=2, ep_length=int(g["ep_length"]),
               device="cuda", buffer_size=64)
    ag.learner.actor.load_state_dict(_sd(g, "actor"))
    ag.learner.fixed_encoder.load_state_dict(_sd(g, "fixed_encoder"))
    return ag


@pytest.mark.gpu
def test_pink_select_action_matches_reference_host_path():
    """Agent.select_action(state, timestep, first_step) over two episodes."""
    g = _g()
    ag = _agent(g)
    seeds = iter(g["noise_seeds"].tolist())
    ag.noise_rng_factory = lambda: np.random.default_rng(next(seeds))
    ep_noise = 0
    for j, (ep, t) in enumerate(g["plan"]):
        a = ag.select_action(g["states"][j], timestep=int(t), first_step=(t == 0))
        if t == 0:
            np.testing.assert_allclose(ag.noise, g["noise"][ep_noise], rtol=1e-6, atol=1e-9)
            ep_noise += 1
        np.testing.assert_allclose(a, g["actions"][j], rtol=0, atol=1e-5, err_msg=f"call {j}")
        assert abs(ag.learner.exploration_noise - g["exploration"][j]) < 1e-7


@pytest.mark.gpu
def test_pink_select_action_matches_reference_device_path():
    """init_episode_noise_device on the reference's spectra + select_action_batch
    (the vectorised loop's path): same noise buffer, actions, decrement."""
    g = _g()
    ag = _agent(g)
    L = int(g["ep_length"])
    for j, (ep, t) in enumerate(g["plan"]):
        if t == 0:
            seed = int(g["noise_seeds"][ep])
            noise = ag.init_episode_noise_device(L, spectrum=_spectrum(seed, 7, L))
            np.testing.assert_allclose(noise.cpu().numpy(), g["noise"][ep], rtol=0, atol=1e-6)
        obs = torch.as_tensor(g["states"][j], device="cuda")
        a = ag.select_action_batch(obs, timestep=torch.tensor([int(t)], device="cuda"))
        np.testing.assert_allclose(a.cpu().numpy(), g["actions"][j], rtol=0, atol=1e-5, err_msg=f"call {j}")
        assert abs(float(ag.learner.exploration_noise_t) - g["exploration"][j]) < 1e-7


@pytest.mark.gpu
@pytest.mark.parametrize("batched", [True, False])
def test_select_action_checkpoint_and_live_on_gpu(batched):
    """tests/golden/select_action.npz: exploration off, checkpoint and live
    nets, through Agent.select_action on the MI355X (1-D and batched states)."""
    from exo_amd.td7 import Agent, Hyperparameters
    g = np.load(f"{GOLDEN}/select_action.npz", allow_pickle=False)
    hp = Hyperparameters(zs_dim=16, enc_hdim=24, critic_hdim=20, actor_hdim=18)
    ag = Agent(80, 7, 1, hp=hp, env_num=2, device="cuda", buffer_size=64)
    for name in ("checkpoint_actor", "checkpoint_encoder", "actor", "fixed_encoder"):
        getattr(ag.learner, name).load_state_dict(_sd(g, name))
    for ckpt, key in ((True, "action_ckpt"), (False, "action_live")):
        if batched:
            a = ag.select_action(g["state"], use_checkpoint=ckpt, use_exploration=False)
        else:
            a = np.stack([ag.select_action(s, use_checkpoint=ckpt, use_exploration=False) for s in g["state"]])
        np.testing.assert_allclose(a, g[key], rtol=0, atol=1e-5, err_msg=key)
        b = ag.select_action_batch(torch.as_tensor(g["state"], device="cuda"), use_checkpoint=ckpt,
                                   use_exploration=False)
        np.testing.assert_allclose(b.cpu().numpy(), g[key], rtol=0, atol=1e-5, err_msg=key)
