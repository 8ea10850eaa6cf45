"""The row-tile-fused TD7 passes (csrc/td7_fused.hip, exo_amd/fused.py) against
the per-layer HIP kernels of the same nets (csrc/td7_dense*.hip, themselves
pinned to fp64 torch per layer by tests/test_td7_dense_gpu.py and end to end to
the reference's golden train() steps by tests/test_td7_full.py).

Both paths round every GEMM operand to bf16 / fp16 at the same points (the
layer inputs and the weights) and accumulate in fp32; they differ in fp32
summation order, which flips an occasional 16-bit rounding of a hidden
activation: the bound is rel = ||fused - per-layer|| / ||per-layer|| <= 1e-2
(observed ~1e-3), elementwise where the output is a noise draw.  Shapes: the
bench's (zs/enc 300, critic/actor 320) and the 256-wide alias; row counts that
are not multiples of the workgroup's rows exercise the masked tail.

fp32 (EXO_FUSED_F32, csrc/td7_fused.h Ty<PREC_F32>: exact products,
v_mfma_f32_16x16x4_f32) against the per-layer fp32 kernels: no rounding
anywhere, only the fp32 summation order differs -- rel <= 2e-5 (observed
~1e-6), the select's actions within 1e-4.
"""
import pytest
import torch

from exo_amd import ops
from exo_amd.td7 import Hyperparameters, TD7Learner

pytestmark = pytest.mark.gpu

REL = 1e-2
REL_F32 = 2e-5


def _tol(precision):
    return REL_F32 if precision == "fp32" else REL


def _rel(x, y):
    return float((x.double() - y.double()).norm() / y.double().norm().clamp_min(1e-30))


def _learner(precision, width):
    torch.manual_seed(3)
    if width is None:
        hp = Hyperparameters()
    elif isinstance(width, dict):  # uneven widths
        hp = Hyperparameters(**width)
    else:
        hp = Hyperparameters(zs_dim=width, enc_hdim=width, critic_hdim=width, actor_hdim=width)
    from exo_amd import fused
    f0 = fused.FUSED_F32
    fused.FUSED_F32 = precision == "fp32"  # read when the learner builds its fused nets
    try:
        L = TD7Learner(80, 7, hp, device="cuda", precision=precision)
    finally:
        fused.FUSED_F32 = f0
    if L.fused is None and isinstance(width, dict):
        pytest.skip("this shape's fused plan does not fit: the per-layer kernels run it "
                    "(test_uneven_widths_probe_or_fall_back)")
    assert L.fused is not None
    # non-trivial target / fixed nets: perturb them away from the live ones
    g = torch.Generator(device="cuda").manual_seed(5)
    with torch.no_grad():
        for m in (L.actor_target, L.critic_target, L.fixed_encoder_target, L.fixed_encoder, L.actor):
            for p in m.parameters():
                p.add_(torch.randn(p.shape, device="cuda", generator=g) * 0.02)
    L.fused.pack_all()
    return L


def _inputs(B, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    s = torch.randn(B, 80, device="cuda", generator=g)
    a = torch.rand(B, 7, device="cuda", generator=g) * 2 - 1
    return s, a


@pytest.mark.parametrize("precision,width,B", [("bf16", None, 1024), ("bf16", None, 1000), ("fp16", None, 1024),
                                               ("bf16", 256, 520), ("fp32", None, 1024), ("fp32", None, 1000),
                                               ("fp32", 256, 520)])
def test_fixed_embeddings_match_per_layer(precision, width, B):
    L = _learner(precision, width)
    s, a = _inputs(B)
    zs, zsa = L.fused.fixed(s, a)
    with torch.no_grad(), ops.matrix_precision(precision):
        zs_ref = L.fixed_encoder.zs(s)
        zsa_ref = L.fixed_encoder.zsa(zs_ref, a)
    torch.cuda.synchronize()
    assert _rel(zs, zs_ref) < _tol(precision), _rel(zs, zs_ref)
    assert _rel(zsa, zsa_ref) < _tol(precision), _rel(zsa, zsa_ref)


# ZS_WIDE: zs_dim well above actor_hdim, where fp32's action output no longer
# fits the overlay region of td7f_target and gets its own
ZS_WIDE = dict(zs_dim=300, enc_hdim=300, critic_hdim=320, actor_hdim=260)


@pytest.mark.parametrize("precision,width,B", [("bf16", None, 1024), ("bf16", None, 1000), ("fp16", None, 1024),
                                               ("bf16", 256, 520), ("fp32", None, 1024), ("fp32", None, 1000),
                                               ("fp32", ZS_WIDE, 520), ("bf16", ZS_WIDE, 520)])
def test_target_chain_matches_per_layer(precision, width, B):
    L = _learner(precision, width)
    ns, _ = _inputs(B, 1)
    z = torch.randn(B, 7, device="cuda", generator=torch.Generator(device="cuda").manual_seed(9))
    sigma0 = float(L.target_policy_noise)
    qt = L.fused.target_heads(ns, z)
    torch.cuda.synchronize()
    assert abs(float(L.target_policy_noise) - (sigma0 - L.policy_noise_decrease)) < 1e-7
    L.target_policy_noise.fill_(sigma0)
    with torch.no_grad(), ops.matrix_precision(precision):
        zs = L.fixed_encoder_target.zs(ns)
        na = ops.noisy_action(L.actor_target(ns, zs), z, L.target_policy_noise, L.policy_noise_decrease,
                              clip=L.hp.noise_clip)
        zsa = L.fixed_encoder_target.zsa(zs, na)
        qt_ref = L.critic_target(ns, na, zsa, zs)
    torch.cuda.synchronize()
    assert qt.shape == qt_ref.shape == (B, 2)
    assert _rel(qt, qt_ref) < _tol(precision), _rel(qt, qt_ref)


@pytest.mark.parametrize("precision,width,n,rt", [("bf16", None, 4096, "1"), ("bf16", None, 1000, "1"),
                                                  ("fp16", None, 4096, "1"), ("bf16", 256, 96, "1"),
                                                  ("bf16", None, 4096, "2"), ("bf16", None, 1000, "2"),
                                                  ("fp16", 256, 96, "2"), ("fp32", None, 4096, "1"),
                                                  ("fp32", None, 1000, "2")])
def test_select_action_matches_per_layer(precision, width, n, rt, monkeypatch):
    """Same Philox draws (the exploration stream's counter is rewound), same
    decrement of exploration_noise (once per env), same clamp; 16 and 32 rows
    per workgroup (EXO_SELECT_RT)."""
    monkeypatch.setenv("EXO_SELECT_RT", rt)
    L = _learner(precision, width)
    obs, _ = _inputs(n, 2)
    rng = L._explore_rng
    st0, sig0 = rng.state.clone(), float(L.exploration_noise_t)
    out = L.fused.select(obs, scale=1.0)
    torch.cuda.synchronize()
    st1, sig1 = rng.state.clone(), float(L.exploration_noise_t)
    rng.state.copy_(st0)
    L.exploration_noise_t.fill_(sig0)
    with torch.no_grad(), ops.matrix_precision(precision):
        ref = ops.noisy_action(L.act(obs), None, L.exploration_noise_t, L.action_noise_decrease * n, rng=rng)
    torch.cuda.synchronize()
    assert torch.equal(rng.state, st1)
    assert abs(float(L.exploration_noise_t) - sig1) < 1e-9
    assert _rel(out, ref) < _tol(precision), _rel(out, ref)
    # actions saturate at +-1 identically where the noise dominates
    assert float((out - ref).abs().max()) < (1e-4 if precision == "fp32" else 0.05)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_fused_trainer_graph_replay_equals_eager(precision):
    """The graph-replayed training loop on the fused passes (fp32 operands:
    the drop-in default; bf16: the bench) trains the nets bit-identically to
    the same loop run eagerly -- both policy-update parities, a target refresh
    (target_update_rate 5), the bench's widths."""
    from exo_amd import VecExoskeletonEnv, fused
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent
    out = []
    for graphs in (False, True):
        torch.manual_seed(7)
        hp = Hyperparameters(batch_size=32, target_update_rate=5)
        env = VecExoskeletonEnv(64, seed=7)
        f0 = fused.FUSED_F32
        fused.FUSED_F32 = True
        try:
            ag = Agent(80, 7, 1, hp=hp, env_num=8, precision=precision, n_envs=64, buffer_size=8192,
                       graph_safe=graphs)
        finally:
            fused.FUSED_F32 = f0
        assert ag.learner.fused is not None
        tr = VecTrainer(env, ag, use_graphs=graphs)
        tr.plan(12)  # graphs: the overlapped pairs (r05) inside the announced run
        for _ in range(12):
            tr.step()
        torch.cuda.synchronize()
        out.append([p.detach().clone() for m in (ag.learner.actor, ag.learner.critic, ag.learner.encoder)
                    for p in m.parameters()])
        if graphs:
            assert tr.graphs, "the graph-replayed trainer captured no graph"
            assert any(k[-1] == "overlap" for k in tr.graphs), "no overlapped pair ran"
    for a, b in zip(*out):
        torch.testing.assert_close(b, a, rtol=0, atol=0)


def test_fp32_select_in_capped_launches_equals_one_launch(monkeypatch):
    """td7f_select with a workgroup cap (wg_cap: the row tiles in
    back-to-back launches of at most cap workgroups, fp32): the same actions
    bit for bit, exploration_noise decremented once and the Philox call
    counter advanced once -- by the last launch's ticket."""
    L = _learner("fp32", None)
    obs, _ = _inputs(4096, 4)
    rng = L._explore_rng
    st0, sig0 = rng.state.clone(), float(L.exploration_noise_t)
    outs, states, sigmas = [], [], []
    monkeypatch.delenv("EXO_SELECT_WG_CAP", raising=False)
    for cap in (0, 100):  # 256 tiles: one launch / launches of 100, 100, 56
        rng.state.copy_(st0)
        L.exploration_noise_t.fill_(sig0)
        outs.append(L.fused.select(obs, scale=1.0, wg_cap=cap))
        torch.cuda.synchronize()
        states.append(rng.state.clone())
        sigmas.append(float(L.exploration_noise_t))
    torch.testing.assert_close(outs[1], outs[0], rtol=0, atol=0)
    assert torch.equal(states[0], states[1]) and not torch.equal(states[0], st0)
    assert sigmas[0] == sigmas[1] < sig0


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_critic_split_launches_equal_one_launch(monkeypatch, precision):
    """td7f_critic_phase (r05): the critic pass as a forward launch beside the
    target chain and a loss + backward launch after it (EXO_CRITIC_SPLIT) --
    the graph-replayed training loop with it and without it: every weight,
    optimiser moment, replay priority and Q bound bit for bit."""
    from exo_amd import VecExoskeletonEnv, fused, td7
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent
    out = []
    for split in (False, True):
        monkeypatch.setattr(td7, "CRITIC_SPLIT", split)
        torch.manual_seed(7)
        env = VecExoskeletonEnv(256, seed=7)
        f0 = fused.FUSED_F32
        fused.FUSED_F32 = True
        try:
            ag = Agent(80, 7, 1, env_num=8, precision=precision, n_envs=256, buffer_size=8192, graph_safe=True)
        finally:
            fused.FUSED_F32 = f0
        tr = VecTrainer(env, ag)
        for _ in range(10):
            tr.step()
        torch.cuda.synchronize()
        L = ag.learner
        st = [p.detach().clone() for m in (L.actor, L.critic, L.encoder) for p in m.parameters()]
        st += [getattr(L, o).m.clone() for o in ("actor_optimizer", "critic_optimizer", "encoder_optimizer")]
        st += [ag.replay_buffer._tree.clone(), L.max.clone(), L.min.clone()]
        out.append(st)
    for i, (a, b) in enumerate(zip(*out)):
        torch.testing.assert_close(b, a, rtol=0, atol=0, msg=f"tensor {i}")


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_uneven_widths_probe_or_fall_back(precision):
    """fp32 with zs_dim well above actor_hdim made td7f_target
    return EINVAL at its first call.  The target pass now overlays its output
    image on X | CATA there, and FusedNets.probe runs every pass once in
    plan-only mode (td7f_probe) when the learner builds them: an inference
    pass that does not fit falls back to the per-layer kernels at
    construction, a gradient pass that does not (here the actor's, 260 wide:
    not a multiple of 16) keeps fused inference and a per-layer update.
    Either way one training step runs and leaves finite weights."""
    import warnings
    from exo_amd import fused
    from exo_amd.td7 import TD7Learner
    torch.manual_seed(4)
    f0 = fused.FUSED_F32
    fused.FUSED_F32 = True
    try:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            L = TD7Learner(80, 7, Hyperparameters(**ZS_WIDE, batch_size=64), device="cuda", precision=precision)
    finally:
        fused.FUSED_F32 = f0
    fell_back = any("per-layer kernels run this network" in str(x.message) for x in w)
    assert (L.fused is None) == fell_back
    print(precision, "per-layer fallback" if L.fused is None else
          f"fused inference, {'fused' if L.fused_train else 'per-layer'} update")
    if L.fused is not None and not L.fused_train:
        assert "EINVAL" in L.fused.train_error
    B = 8 * 64
    g = torch.Generator(device="cuda").manual_seed(2)
    s, ns = torch.randn(B, 80, device="cuda", generator=g), torch.randn(B, 80, device="cuda", generator=g)
    a = torch.rand(B, 7, device="cuda", generator=g) * 2 - 1
    r, nd = torch.rand(B, 1, device="cuda", generator=g), torch.ones(B, 1, device="cuda")
    L.update(s, a, ns, r, nd, update_actor=True)
    torch.cuda.synchronize()
    for m in (L.actor, L.critic, L.encoder):
        assert all(torch.isfinite(p).all() for p in m.parameters())
    if L.fused is not None:
        qt = L.fused.target_heads(ns, torch.zeros(B, 7, device="cuda"))
        zs, zsa = L.fused.fixed(s, a)
        torch.cuda.synchronize()
        assert torch.isfinite(qt).all() and torch.isfinite(zs).all() and torch.isfinite(zsa).all()


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_select_row_tiles_argument(precision):
    """td7f_select's rt argument (r05: the training loop asks for 32-row tiles
    at 4,096 envs): 16- and 32-row tiles draw the same noise per row and agree
    to the fused passes' bound (another fp32 summation order flips an
    occasional 16-bit rounding of a hidden activation), and both match the
    per-layer path (test_select_action_matches_per_layer[..-2])."""
    L = _learner(precision, None)
    s, _ = _inputs(4096, 11)
    sigma = float(L.exploration_noise_t)
    outs = []
    st0 = L._explore_rng.state.clone()
    for rt in (1, 2):
        L.exploration_noise_t.fill_(sigma)
        L._explore_rng.state.copy_(st0)  # the same noise draws
        outs.append(L.fused.select(s, scale=1.0, rt=rt))
    torch.cuda.synchronize()
    assert _rel(outs[1], outs[0]) < REL, _rel(outs[1], outs[0])
    assert float((outs[1] - outs[0]).abs().max()) < 2e-2


@pytest.mark.parametrize("precision,rt,cap", [("bf16", 1, 0), ("bf16", 2, 0), ("fp16", 2, 0), ("fp32", 1, 0),
                                              ("fp32", 1, 100)])
def test_split_select_equals_one_launch(precision, rt, cap):
    """td7f_select_part (r06): the fixed encoder's zs half (mode 1, into the
    zs image) then the actor half from it (mode 2) -- the actions bit for bit
    those of the one-launch td7f_select at the same row tiles, the Philox call
    counter and exploration_noise advanced once (by the actor half only), the
    zs half alone leaving both untouched; with the fp32 workgroup cap too."""
    L = _learner(precision, None)
    obs, _ = _inputs(4096, 13)
    rng = L._explore_rng
    st0, sig0 = rng.state.clone(), float(L.exploration_noise_t)
    one = L.fused.select(obs, scale=1.0, rt=rt, wg_cap=cap)
    torch.cuda.synchronize()
    st1, sig1 = rng.state.clone(), float(L.exploration_noise_t)
    rng.state.copy_(st0)
    L.exploration_noise_t.fill_(sig0)
    img = L.fused.select_zs(obs, rt=rt, wg_cap=cap)
    torch.cuda.synchronize()
    assert torch.equal(rng.state, st0) and float(L.exploration_noise_t) == sig0
    two = L.fused.select(obs, scale=1.0, rt=rt, wg_cap=cap, zs_img=img)
    torch.cuda.synchronize()
    torch.testing.assert_close(two, one, rtol=0, atol=0)
    assert torch.equal(rng.state, st1) and float(L.exploration_noise_t) == sig1
