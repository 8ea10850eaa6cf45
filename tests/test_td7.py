"""TD7 update math (exo_amd.td7.TD7Learner, device-agnostic torch) against the
reference's golden train() steps (tests/golden/td7_small.npz: reduced widths,
injected batch and target-policy noise).  fp32 on CPU: tolerance 1e-5 rel /
1e-6 abs on every parameter after each step."""
import numpy as np
import pytest
import torch

from helpers import GOLDEN
from exo_amd.td7 import Hyperparameters, TD7Learner


def _golden():
    return np.load(f"{GOLDEN}/td7_small.npz", allow_pickle=False)


def _learner(g, device="cpu"):
    zs, enc, crit, act, bs, E = [int(x) for x in g["hp"]]
    hp = Hyperparameters(zs_dim=zs, enc_hdim=enc, critic_hdim=crit, actor_hdim=act, batch_size=bs)
    torch.manual_seed(0)
    L = TD7Learner(80, 7, hp, learning_steps=int(g["learning_steps"]), device=device, fused_adam=False)
    return L


def _sd(g, prefix):
    return {k[len(prefix) + 1:]: torch.tensor(g[k]) for k in g.files if k.startswith(prefix + ".")}


def test_seeded_init_matches_reference():
    g = _golden()
    L = _learner(g)
    for name in ("actor", "critic", "encoder"):
        ref = _sd(g, f"init_{name}")
        for k, v in getattr(L, name).state_dict().items():
            torch.testing.assert_close(v, ref[k], rtol=0, atol=0)


@pytest.mark.parametrize("device", ["cpu"])
def test_two_train_steps_match_reference(device):
    g = _golden()
    L = _learner(g, device)
    for step in range(2):
        b = [torch.tensor(g[f"batch{step}_{k}"], device=device) for k in
             ("state", "action", "next_state", "reward", "not_done")]
        noise = torch.tensor(g[f"batch{step}_noise"], device=device)
        prio = L.update(*b, noise=noise)
        np.testing.assert_allclose(prio.cpu().numpy(), g[f"priority{step}"], rtol=1e-5, atol=1e-6)
        for name in ("actor", "critic", "encoder"):
            ref = _sd(g, f"step{step}_{name}")
            for k, v in getattr(L, name).state_dict().items():
                np.testing.assert_allclose(v.cpu().numpy(), ref[k].numpy(), rtol=1e-5, atol=1e-6,
                                           err_msg=f"step {step} {name}.{k}")
        assert abs(float(L.max) - g[f"step{step}_max"]) <= 1e-5 * max(1, abs(g[f"step{step}_max"]))
        assert abs(float(L.min) - g[f"step{step}_min"]) <= 1e-5 * max(1, abs(g[f"step{step}_min"]))
        assert abs(float(L.target_policy_noise) - g[f"step{step}_target_policy_noise"]) < 1e-7


def test_target_update_schedule():
    hp = Hyperparameters(zs_dim=8, enc_hdim=8, critic_hdim=8, actor_hdim=8, batch_size=4, target_update_rate=3)
    L = TD7Learner(80, 7, hp, device="cpu", fused_adam=False)
    b = [torch.randn(4, 80), torch.rand(4, 7) * 2 - 1, torch.randn(4, 80), torch.rand(4, 1), torch.ones(4, 1)]
    for i in range(1, 7):
        L.update(*b)
        refreshed = L.maybe_update_targets()
        assert refreshed == (i % 3 == 0)
        if refreshed:
            for p, q in zip(L.critic.parameters(), L.critic_target.parameters()):
                assert torch.equal(p, q)
            assert float(L.max_target) == float(L.max)


def test_select_action_matches_reference_pink_variant():
    g = np.load(f"{GOLDEN}/select_action.npz", allow_pickle=False)
    hp = Hyperparameters(zs_dim=16, enc_hdim=24, critic_hdim=20, actor_hdim=18)
    L = TD7Learner(80, 7, hp, device="cpu", fused_adam=False)
    for name in ("checkpoint_actor", "checkpoint_encoder", "actor", "fixed_encoder"):
        getattr(L, name).load_state_dict(_sd(g, name))
    st = torch.tensor(g["state"])
    np.testing.assert_allclose(L.act(st, use_checkpoint=True).numpy(), g["action_ckpt"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(L.act(st, use_checkpoint=False).numpy(), g["action_live"], rtol=1e-6, atol=1e-6)


def test_pink_noise_statistics():
    from exo_amd.pink import powerlaw_psd_gaussian
    x = powerlaw_psd_gaussian(1.0, (7, 4096), rng=np.random.default_rng(0))
    assert x.shape == (7, 4096)
    assert abs(x.std() - 1) < 0.2
    # 1/f: low-frequency power dominates
    p = np.abs(np.fft.rfft(x, axis=-1)) ** 2
    assert p[:, 1:20].mean() > 10 * p[:, 1000:1200].mean()


@pytest.mark.gpu
def test_two_train_steps_match_reference_on_gpu():
    """Same golden steps with the nets on the MI355X (fp32, hipBLASLt GEMMs)."""
    g = _golden()
    L = _learner(g, "cpu")
    L2 = TD7Learner(80, 7, L.hp, learning_steps=int(g["learning_steps"]), device="cuda")
    for name in ("actor", "critic", "encoder", "actor_target", "critic_target", "fixed_encoder",
                 "fixed_encoder_target"):
        getattr(L2, name).load_state_dict(getattr(L, name).state_dict())
    for step in range(2):
        b = [torch.tensor(g[f"batch{step}_{k}"], device="cuda") for k in
             ("state", "action", "next_state", "reward", "not_done")]
        prio = L2.update(*b, noise=torch.tensor(g[f"batch{step}_noise"], device="cuda"))
        np.testing.assert_allclose(prio.cpu().numpy(), g[f"priority{step}"], rtol=1e-4, atol=1e-5)
        for name in ("actor", "critic", "encoder"):
            ref = _sd(g, f"step{step}_{name}")
            for k, v in getattr(L2, name).state_dict().items():
                np.testing.assert_allclose(v.cpu().numpy(), ref[k].numpy(), rtol=1e-4, atol=1e-5,
                                           err_msg=f"step {step} {name}.{k}")


@pytest.mark.gpu
def test_agent_train_step_through_lap_kernels():
    from exo_amd import td7
    td7.smoke()


def test_critic_state_dict_uses_reference_names():
    from exo_amd.td7 import Critic
    c = Critic(80, 7, 16, 20)
    sd = c.state_dict()
    assert sorted(sd) == sorted(f"{n}.{p}" for n in ("q01", "q1", "q2", "q3", "q02", "q4", "q5", "q6")
                                for p in ("weight", "bias"))
    c2 = Critic(80, 7, 16, 20)
    c2.load_state_dict(sd)
    for a, b in zip(c.parameters(), c2.parameters()):
        assert torch.equal(a, b)


def test_loads_shipped_reference_checkpoint():
    """Simulation/AGENT_NNS/[0,0,0,1] (reference, weights_only): the nets load
    with the reference's names and the Pink-noise widths (actor 300)."""
    import os
    path = "/root/reference/Simulation/AGENT_NNS/[0,0,0,1]/[0,0,0,1]"
    if not os.path.exists(path + "_actor"):
        pytest.skip("reference checkpoints not present")
    from exo_amd.td7 import Actor, Critic, Encoder
    a, c, e = Actor(80, 7, 300, 300), Critic(80, 7, 300, 320), Encoder(80, 7, 300, 300)
    a.load_state_dict(torch.load(path + "_actor", map_location="cpu", weights_only=True))
    c.load_state_dict(torch.load(path + "_critic", map_location="cpu", weights_only=True))
    e.load_state_dict(torch.load(path + "_encoder", map_location="cpu", weights_only=True))
    s = torch.randn(4, 80)
    act = a(s, e.zs(s))
    assert act.shape == (4, 7) and torch.all(act.abs() <= 1)
    q = c(s, act, e.zsa(e.zs(s), act), e.zs(s))
    assert q.shape == (4, 2) and torch.isfinite(q).all()


@pytest.mark.gpu
def test_flat_adam_matches_torch_adam():
    """FlatAdam (td7_adam_step) vs torch.optim.Adam on the same net and
    gradients, over several steps; state_dict round trip keeps the moments."""
    import copy

    import torch.nn.functional as F
    from exo_amd.td7 import Encoder, FlatAdam
    torch.manual_seed(0)
    net = Encoder(80, 7, 64, 96, F.elu).cuda()
    ref = copy.deepcopy(net)
    opt = FlatAdam(net, lr=3e-4, weight_decay=1e-7)
    opt_ref = torch.optim.Adam(ref.parameters(), lr=3e-4, weight_decay=1e-7)
    for it in range(5):
        x = torch.randn(128, 80, device="cuda")
        a = torch.randn(128, 7, device="cuda")
        for m, o in ((net, opt), (ref, opt_ref)):
            o.zero_grad(set_to_none=True)
            zs = m.zs(x)
            (m.zsa(zs, a).square().mean() + zs.abs().mean()).backward()
        for p, q in zip(net.parameters(), ref.parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-6)
        opt.step()
        opt_ref.step()
        for p, q in zip(net.parameters(), ref.parameters()):
            torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    assert float(opt._step) == 5.0
    sd = opt.state_dict()
    opt2 = FlatAdam(copy.deepcopy(net), lr=3e-4, weight_decay=1e-7)
    opt2.load_state_dict(sd)
    torch.testing.assert_close(opt2.m, opt.m)
    torch.testing.assert_close(opt2.v, opt.v)
    assert float(opt2._step) == 5.0
    # the reference's torch Adam loads a FlatAdam state_dict
    opt_ref.load_state_dict(sd)


@pytest.mark.gpu
def test_device_pink_noise_matches_numpy_and_statistics():
    """powerlaw_psd_gaussian_device: the deterministic half (masking,
    normalisation, irfft) equals the numpy path on the same spectra; the
    generated sequences have unit variance; the batched Pink select_action
    adds column t of the episode noise to every env."""
    from exo_amd.pink import irfft_reference, powerlaw_psd_gaussian_device
    from exo_amd.td7 import Agent, Hyperparameters
    rng = np.random.default_rng(0)
    for n in (341, 344):
        sr, si = rng.normal(size=(7, n // 2 + 1)), rng.normal(size=(7, n // 2 + 1))
        dev = powerlaw_psd_gaussian_device(1.0, 7, n, "cuda", spectrum=(sr, si)).cpu().numpy()
        np.testing.assert_allclose(dev, irfft_reference(sr, si, 1.0, n), rtol=1e-5, atol=1e-6)
    big = powerlaw_psd_gaussian_device(1.0, 4096, 344, "cuda").cpu().numpy()
    assert abs(big.mean()) < 0.05 and abs(big.std() - 1.0) < 0.05
    hp = Hyperparameters(zs_dim=32, enc_hdim=32, critic_hdim=32, actor_hdim=32, batch_size=16)
    ag = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=1024, ep_length=50)
    noise = ag.init_episode_noise_device(50).clone()
    assert float(noise.abs().max()) == pytest.approx(float(ag.learner.exploration_noise_t), rel=1e-6)
    obs = torch.randn(64, 80, device="cuda")
    t = torch.tensor([7], device="cuda")
    a = ag.select_action_batch(obs, timestep=t)
    ref = (ag.learner.act(obs) + noise[:, 7][None, :]).clamp(-1, 1)
    torch.testing.assert_close(a, ref, rtol=0, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_reduced_precision_train_steps_track_fp32(precision):
    """BASELINE configs[1] ("TD7 bf16") / configs[4] ("fp16 MFMA"): the golden
    steps with bf16 / fp16 MFMA operands stay within the rounding error of the
    fp32 reference (priorities 2e-2, parameters 1e-3 after two Adam steps)."""
    g = _golden()
    L = _learner(g, "cpu")
    L2 = TD7Learner(80, 7, L.hp, learning_steps=int(g["learning_steps"]), device="cuda", precision=precision)
    for name in ("actor", "critic", "encoder", "actor_target", "critic_target", "fixed_encoder",
                 "fixed_encoder_target"):
        getattr(L2, name).load_state_dict(getattr(L, name).state_dict())
    for step in range(2):
        b = [torch.tensor(g[f"batch{step}_{k}"], device="cuda") for k in
             ("state", "action", "next_state", "reward", "not_done")]
        prio = L2.update(*b, noise=torch.tensor(g[f"batch{step}_noise"], device="cuda"))
        np.testing.assert_allclose(prio.cpu().numpy(), g[f"priority{step}"], rtol=2e-2, atol=2e-2)
        for name in ("actor", "critic", "encoder"):
            ref = _sd(g, f"step{step}_{name}")
            for k, v in getattr(L2, name).state_dict().items():
                np.testing.assert_allclose(v.cpu().numpy(), ref[k].numpy(), rtol=0, atol=1e-3,
                                           err_msg=f"step {step} {name}.{k}")


def test_critic_optimizer_state_interchanges_with_reference_layout():
    """The critic's FlatAdam state_dict uses the reference Critic's 16
    per-head parameters (q01 ... q3, q02 ... q6, Agent/TD7_multi_agent.py:109-121),
    so a reference-saved _critic_optimizer loads here and ours loads into the
    reference's torch.optim.Adam (the stacked heads had 8)."""
    import torch.nn as nn
    from exo_amd.td7 import Critic, FlatAdam

    class RefCritic(nn.Module):  # the reference's parameter layout (names and order)
        def __init__(self, s, a, zs, h):
            super().__init__()
            self.q01, self.q1, self.q2, self.q3 = (nn.Linear(s + a, h), nn.Linear(2 * zs + h, h), nn.Linear(h, h),
                                                   nn.Linear(h, 1))
            self.q02, self.q4, self.q5, self.q6 = (nn.Linear(s + a, h), nn.Linear(2 * zs + h, h), nn.Linear(h, h),
                                                   nn.Linear(h, 1))

    torch.manual_seed(0)
    c = Critic(80, 7, 16, 20)
    ref = RefCritic(80, 7, 16, 20)
    ref.load_state_dict(c.state_dict())
    opt_ref = torch.optim.Adam(ref.parameters(), lr=3e-4, weight_decay=1e-7)
    for _ in range(3):
        opt_ref.zero_grad()
        sum((p * torch.randn_like(p)).sum() for p in ref.parameters()).backward()
        opt_ref.step()
    ours = FlatAdam(c, lr=3e-4, weight_decay=1e-7, layout=Critic.optimizer_layout())
    ours.load_state_dict(opt_ref.state_dict())
    ref_params = list(ref.parameters())
    ref_state = opt_ref.state_dict()["state"]
    for j, p in enumerate(c.parameters()):
        for ref_i, h in Critic.optimizer_layout()[j]:
            assert ref_params[ref_i].shape == p[h].shape
            torch.testing.assert_close(ours.state[p]["exp_avg"][h], ref_state[ref_i]["exp_avg"], rtol=0, atol=0)
            torch.testing.assert_close(ours.state[p]["exp_avg_sq"][h], ref_state[ref_i]["exp_avg_sq"], rtol=0, atol=0)
    assert float(ours._step) == 3.0
    # and back: our state_dict loads into the reference's Adam unchanged
    sd = ours.state_dict()
    assert sorted(sd["state"]) == list(range(16)) and sd["param_groups"][0]["params"] == list(range(16))
    opt_ref2 = torch.optim.Adam(RefCritic(80, 7, 16, 20).parameters(), lr=3e-4, weight_decay=1e-7)
    opt_ref2.load_state_dict(sd)
    for i in range(16):
        torch.testing.assert_close(opt_ref2.state_dict()["state"][i]["exp_avg"], ref_state[i]["exp_avg"])
