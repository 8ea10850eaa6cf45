"""In-kernel random numbers (ops.DeviceRNG; csrc/philox.h): the target-policy /
exploration noise of td7_noisy_action_rng and the replay uniforms of
lap_sample_gather_rng against a numpy restatement of Philox4x32-10 (Salmon et
al., SC'11) with the same key / counter layout, plus the statistics the
reference's torch.randn / torch.rand draws have."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

M32 = np.uint64(0xFFFFFFFF)


def philox(j, call, tag, seed):
    """Philox4x32-10 blocks for counters (j, call lo, call hi, tag), key seed -> [n, 4] uint32."""
    j = np.asarray(j, dtype=np.uint64)
    c = [j & M32, np.full_like(j, call & 0xFFFFFFFF), np.full_like(j, call >> 32), np.full_like(j, tag)]
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64(seed >> 32)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        n0 = (p1 >> np.uint64(32)) ^ c[1] ^ k0
        n2 = (p0 >> np.uint64(32)) ^ c[3] ^ k1
        c = [n0 & M32, p1 & M32, n2 & M32, p0 & M32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return np.stack(c, 1).astype(np.uint32)


def test_noisy_action_rng_draws_box_muller_normals_of_philox():
    from exo_amd import ops
    rng = ops.DeviceRNG(torch.device("cuda"), 7)
    n = 20001
    a = torch.zeros(n, device="cuda")
    sigma = torch.tensor(0.1, device="cuda")
    outs = [ops.noisy_action(a, None, sigma, 0.0, rng=rng) for _ in range(2)]
    torch.cuda.synchronize()
    assert int(rng.state[0]) == 2 and int(rng.state[1]) == 0
    for call, out in enumerate(outs):
        r = philox(np.arange((n + 1) // 2), call, 7, rng.seed).astype(np.float64)
        u1 = (np.floor(r[:, 0] / 256) + 1) * 2.0 ** -24
        u2 = np.floor(r[:, 1] / 256) * 2.0 ** -24
        rad = np.sqrt(-2 * np.log(u1))
        z = np.stack([rad * np.cos(2 * np.pi * u2), rad * np.sin(2 * np.pi * u2)], 1).reshape(-1)[:n]
        np.testing.assert_allclose(out.cpu().numpy(), np.clip(0.1 * z, -1, 1), rtol=0, atol=2e-6)
    z = outs[0].cpu().numpy() / 0.1
    assert abs(z.mean()) < 0.03 and abs(z.std() - 1) < 0.02
    assert not torch.equal(outs[0], outs[1])


def test_noisy_action_rng_clip_scale_and_sigma_decay():
    from exo_amd import ops
    rng = ops.DeviceRNG(torch.device("cuda"), 8)
    a = torch.rand(4096, 7, device="cuda") * 2 - 1
    sigma = torch.tensor(0.5, device="cuda")
    out = ops.noisy_action(a, None, sigma, 0.125, clip=0.3, scale=2.0, rng=rng)
    assert float(sigma) == 0.375
    assert float(out.abs().max()) <= 2.0
    e = out / 2 - a
    inside = (a.abs() < 0.69)  # far from the action clamp: the noise is the clipped draw
    assert float(e[inside].abs().max()) <= 0.3 + 1e-6


def test_lap_sample_rng_uses_the_philox_uniforms():
    """lap_sample_gather_rng picks exactly the indices lap_sample gives for the
    Philox uniforms of its draw indices; the call counter advances per launch."""
    from exo_amd.replay import LAP
    E, C, batch = 4, 64, 16
    lap = LAP(80, 7, "cuda", E, max_size=C, batch_size=batch)
    assert lap.device_rng
    n = 200
    g = torch.Generator(device="cuda").manual_seed(2)
    strata = torch.randint(0, E, (n,), device="cuda", dtype=torch.int32, generator=g)
    obs = torch.randn(n, 80, device="cuda", generator=g)
    lap.add_batch(obs, torch.zeros(n, 7, device="cuda"), obs, torch.zeros(n, device="cuda"),
                  torch.zeros(n, dtype=torch.uint8, device="cuda"), strata)
    prio = torch.randint(1, 9, (E * C,), device="cuda", generator=g).float()
    lap.update_priority(prio, ind=torch.arange(C, dtype=torch.int32, device="cuda").repeat(E, 1).contiguous())
    for call in range(3):
        lap.sample()
        r = philox(np.arange(E * batch), call, lap._rng.tag, lap._rng.seed)
        u = (np.floor(r[:, 0].astype(np.float64) / 256) * 2.0 ** -24).astype(np.float32).reshape(E, batch)
        np.testing.assert_array_equal(lap.ind.cpu().numpy(), lap.sample_indices(torch.as_tensor(u)).cpu().numpy())
    torch.cuda.synchronize()
    assert int(lap._rng.state[0]) == 3 and int(lap._rng.state[1]) == 0
