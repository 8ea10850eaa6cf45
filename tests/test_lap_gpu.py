"""HIP LAP sum-tree kernels (csrc/lap.hip) against the reference's LAP.sample
indices (tests/golden/lap_cases.npz: integer priorities -> exact sums, so the
tree descent must return exactly searchsorted_left(cumsum(p), u*sum))."""
import numpy as np
import pytest
import torch

from helpers import GOLDEN

pytestmark = pytest.mark.gpu


def _lap(E, size, batch):
    from exo_amd.replay import LAP
    return LAP(80, 7, "cuda", E, max_size=size, batch_size=batch)


def _set_priorities(lap, prio):
    E, C = prio.shape
    idx = torch.arange(C, dtype=torch.int32, device="cuda").repeat(E, 1).contiguous()
    lap.update_priority(torch.as_tensor(prio.reshape(-1), device="cuda"), ind=idx)


def test_sample_matches_reference_searchsorted():
    g = np.load(f"{GOLDEN}/lap_cases.npz", allow_pickle=False)
    prio, size, u, ref = g["priority"], int(g["size"]), g["u"], g["index"]
    E, C = prio.shape
    lap = _lap(E, C, u.shape[1])
    _set_priorities(lap, prio)
    lap.size_s.fill_(size)
    idx = lap.sample_indices(torch.as_tensor(u)).cpu().numpy()
    np.testing.assert_array_equal(idx, ref)
    # totals are exact for integer priorities
    np.testing.assert_array_equal(lap.totals.cpu().numpy(), prio.sum(1))
    # brute-force reference semantics for many uniforms
    uu = np.random.default_rng(0).uniform(0, 1, (E, 512)).astype(np.float32)
    idx = lap.sample_indices(torch.as_tensor(uu)).cpu().numpy()
    for s in range(E):
        cs = np.cumsum(prio[s, :size].astype(np.float32))
        want = np.searchsorted(cs, uu[s] * cs[-1], side="left")
        np.testing.assert_array_equal(idx[s], want)


def test_update_last_duplicate_wins_and_max_priority():
    lap = _lap(2, 16, 4)
    _set_priorities(lap, np.ones((2, 16), dtype=np.float32))
    idx = torch.tensor([[5, 5, 7, 5], [0, 1, 2, 3]], dtype=torch.int32, device="cuda")
    pr = torch.tensor([2.0, 3.0, 4.0, 1.5, 9.0, 1.0, 1.0, 1.0], device="cuda")
    lap.update_priority(pr, ind=idx)
    p = lap.priority.cpu().numpy()
    assert p[0, 5] == 1.5 and p[0, 7] == 4.0 and p[1, 0] == 9.0
    assert lap.max_priority == 9.0
    np.testing.assert_allclose(lap.totals.cpu().numpy(), p.sum(1), rtol=1e-6)
    lap.update_priority(torch.ones(8, device="cuda"), ind=torch.tensor([[0, 0, 0, 0], [0, 0, 0, 0]],
                                                                        dtype=torch.int32, device="cuda"))
    assert lap.max_priority == 9.0          # max(max_priority, batch max)
    lap.reset_max_priority()
    assert lap.max_priority == 4.0          # max over the leaves (:120)


def test_add_batch_rings_and_trash_row():
    lap = _lap(4, 8, 4)
    n = 12
    strata = torch.arange(n, device="cuda", dtype=torch.int32) % 4
    active = torch.ones(n, dtype=torch.bool, device="cuda")
    active[5] = False  # stratum 1 gets 2 items this step
    obs = torch.arange(n, device="cuda", dtype=torch.float32)[:, None].repeat(1, 80)
    act = torch.zeros(n, 7, device="cuda")
    for step in range(3):
        lap.add_batch(obs + 100 * step, act, obs, torch.ones(n, device="cuda"), torch.zeros(n, device="cuda"),
                      strata, active)
    ptr = lap.ptr_s.cpu().numpy()
    size = lap.size_s.cpu().numpy()
    np.testing.assert_array_equal(size, [8, 6, 8, 8])          # 9 adds wrap a ring of 8
    np.testing.assert_array_equal(ptr, [1, 6, 1, 1])
    st = lap.state.cpu().numpy()
    assert st[1, :6, 0].tolist() == [1, 9, 101, 109, 201, 209]
    assert st[0, 0, 0] == 208 and st[0, 1, 0] == 4            # slot 0 overwritten by the 9th add
    p = lap.priority.cpu().numpy()
    assert np.all(p[1, :6] == 1.0) and np.all(p[1, 6:] == 0.0)


def test_sampling_frequencies_follow_priorities():
    lap = _lap(1, 4, 4096)
    _set_priorities(lap, np.array([[1.0, 3.0, 0.0, 4.0]], dtype=np.float32))
    lap.size_s.fill_(4)
    counts = np.zeros(4)
    for _ in range(20):
        lap.sample()
        counts += np.bincount(lap.ind.cpu().numpy().ravel(), minlength=4)
    f = counts / counts.sum()
    np.testing.assert_allclose(f, [1 / 8, 3 / 8, 0, 4 / 8], atol=0.01)


def test_reference_single_add_pointer_semantics():
    """LAP.add (:59-63): env 0's first write lands one slot behind the others."""
    lap = _lap(3, 10, 2)
    for step in range(2):
        for e in range(3):
            lap.add(np.full(80, 10 * step + e), np.zeros(7), np.zeros(80), 1.0, False, e)
    st = lap.state.cpu().numpy()[:, :, 0]
    assert st[0, 0] == 0 and st[1, 1] == 1 and st[2, 1] == 2 and st[0, 1] == 10 and st[1, 2] == 11
    assert lap.ptr == 2 and lap.size == 2 and lap.count == 6


def test_sample_gathers_the_rows_of_its_indices():
    """lap_sample_gather: the returned batch is the storage rows at lap.ind
    (stratum-major), with action scaled and not_done = 1 - done as stored."""
    lap = _lap(4, 64, 16)
    n = 200
    g = torch.Generator(device="cuda").manual_seed(1)
    strata = torch.randint(0, 4, (n,), device="cuda", dtype=torch.int32, generator=g)
    for step in range(3):
        obs = torch.randn(n, 80, device="cuda", generator=g)
        act = torch.rand(n, 7, device="cuda", generator=g) * 2 - 1
        done = (torch.rand(n, device="cuda", generator=g) < 0.3).to(torch.uint8)
        lap.add_batch(obs, act, obs + 1, torch.randn(n, device="cuda", generator=g), done, strata)
    s, a, ns, r, nd = lap.sample()
    idx = lap.ind.long()
    rows = (torch.arange(4, device="cuda")[:, None] * 65 + idx).reshape(-1)
    torch.testing.assert_close(s, lap.state.view(-1, 80)[rows], rtol=0, atol=0)
    torch.testing.assert_close(a, lap.action.view(-1, 7)[rows], rtol=0, atol=0)
    torch.testing.assert_close(ns, lap.next_state.view(-1, 80)[rows], rtol=0, atol=0)
    torch.testing.assert_close(r, lap.reward.view(-1, 1)[rows], rtol=0, atol=0)
    torch.testing.assert_close(nd, lap.not_done.view(-1, 1)[rows], rtol=0, atol=0)
    assert int(idx.max()) < 64 and set(torch.unique(nd).tolist()) <= {0.0, 1.0}
    sizes = lap.size_s.cpu().numpy()
    assert all(int(idx[k].max()) < sizes[k] for k in range(4))


def test_sample_matches_reference_at_full_depth():
    """tests/golden/lap_full.npz: the reference's LAP.sample at max_size 2.5e5
    (all 18 tree levels active, 180,000 filled rows) with a nonzero leaf at
    slot == size in strata 1-2 (the single-add pointer quirk, :59-61): the
    descent is scaled by the prefix total over [0, size), so the indices match
    searchsorted_left(cumsum(priority[:size]), u * total) exactly."""
    g = np.load(f"{GOLDEN}/lap_full.npz", allow_pickle=False)
    prio, size, u, ref = g["priority"].astype(np.float32), int(g["size"]), g["u"], g["index"]
    E, C = prio.shape
    lap = _lap(E, C, u.shape[1])
    assert lap._cap == 1 << 18
    _set_priorities(lap, prio)
    lap.size_s.fill_(size)
    np.testing.assert_array_equal(lap.totals.cpu().numpy(), prio.sum(1))  # root includes slot == size
    idx = lap.sample_indices(torch.as_tensor(u)).cpu().numpy()
    np.testing.assert_array_equal(idx, ref)
    assert idx.max() < size
    # the fused sample + gather kernel descends identically: tag every stored
    # row with its slot and check the gathered rows
    slots = torch.arange(C + 1, device="cuda", dtype=torch.float32)
    lap.reward[:, :, 0] = slots
    lap.state[:, :, 0] = slots
    lap.next_state[:, :, 1] = -slots
    lap.device_rng = False
    lap._u.copy_(torch.as_tensor(u))
    lap._u.uniform_ = lambda: lap._u  # keep the injected uniforms
    s, a, s2, r, nd = lap.sample()
    got = lap.ind.cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(r.cpu().numpy().reshape(E, -1), ref.astype(np.float32))
    np.testing.assert_array_equal(s[:, 0].cpu().numpy().reshape(E, -1), ref.astype(np.float32))
    np.testing.assert_array_equal(s2[:, 1].cpu().numpy().reshape(E, -1), -ref.astype(np.float32))


def test_sample_never_returns_the_slot_at_size():
    """Single-add pointer quirk: the newest transition of strata 1.. sits at
    slot == size and carries max_priority; the reference never samples it
    until size grows past it."""
    lap = _lap(3, 64, 256)
    for step in range(5):
        for e in range(3):
            lap.add(np.zeros(80), np.zeros(7), np.zeros(80), 0.0, False, tremor_num=e)
    assert lap.size == 5
    p = lap.priority.cpu().numpy()
    assert p[1, 5] == 1.0 and p[2, 5] == 1.0 and p[0, 5] == 0.0  # written past size
    idx = lap.sample_indices(torch.rand(3, 256, device="cuda")).cpu().numpy()
    assert idx.max() <= 4
    # with uniform priorities every filled slot < size is drawn: stratum 0
    # holds slots 0-4, strata 1-2 slots 1-5 (their slot 0 was never written)
    assert set(np.unique(idx[0])) == {0, 1, 2, 3, 4}
    assert set(np.unique(idx[1])) == set(np.unique(idx[2])) == {1, 2, 3, 4}


@pytest.mark.parametrize("fused", [True, False])
def test_add_batch_ref_equals_sequential_reference_adds(fused):
    """lap_store_batch_ref (fused: the one-launch lap_store_batch_ref_fused) ==
    LAP.add (:49-63) called once per active row in row order: stored
    transitions, leaves, sums, the shared pointer and size -- random strata
    (several rows per stratum), random active masks (overwrites of one slot by
    two adds of a stratum between pointer advances: the later add wins), a
    pointer that wraps the capacity."""
    rng = np.random.default_rng(3)
    E, C, N = 4, 40, 19
    seq, vec = _lap(E, C, 4), _lap(E, C, 4)
    vec.ref_insert_fused = fused
    for step in range(30):
        st = rng.normal(size=(N, 80)).astype(np.float32)
        nx = rng.normal(size=(N, 80)).astype(np.float32)
        ac = rng.uniform(-1, 1, (N, 7)).astype(np.float32)
        rw = rng.normal(size=N).astype(np.float32)
        dn = rng.random(N) < 0.1
        strata = rng.integers(0, E, N).astype(np.int32)
        active = rng.random(N) < (0.3 if step % 3 else 0.9)
        if step % 7 == 3:  # a max_priority other than 1 for the new leaves
            pr = torch.full((E * 4,), 1.0 + step, device="cuda")
            for lap in (seq, vec):
                lap.update_priority(pr, ind=torch.zeros((E, 4), dtype=torch.int32, device="cuda"))
        for i in np.flatnonzero(active):
            seq.add(st[i], ac[i], nx[i], float(rw[i]), bool(dn[i]), tremor_num=int(strata[i]))
        T = lambda a: torch.as_tensor(a, device="cuda")  # noqa: E731
        vec.add_batch_ref(T(st), T(ac), T(nx), T(rw), T(dn), T(strata), T(active))
        torch.cuda.synchronize()
        assert vec.ref_pointer() == (seq.ptr, seq.count, seq.size), step
        for name in ("state", "action", "next_state", "reward", "not_done"):
            torch.testing.assert_close(getattr(vec, name)[:, :C], getattr(seq, name)[:, :C], rtol=0, atol=0)
        torch.testing.assert_close(vec._tree, seq._tree, rtol=0, atol=0)
        assert torch.equal(vec.size_s, seq.size_s)
    assert seq.count > 2 * C  # the pointer wrapped


@pytest.mark.parametrize("E,C,N", [(8, 5000, 10_000), (8, 30_000, 4096), (5, 3000, 9001)])
def test_fused_ref_insert_equals_three_launch_insert(E, C, N):
    """lap_store_batch_ref_fused (one launch, r04) against the three-launch
    lap_store_batch_ref (pinned to the sequential adds above) at the rollout's
    sizes: several 4,096-row chunks (a stratum's last row of a chunk decided by
    the next chunk), more copy parts than one, non-integer priorities already
    in the tree, masks with whole runs of done envs, ring wrap-around; the
    storage, every tree node, the shared pointer and the sizes bit for bit,
    and every internal node exactly left + right."""
    rng = np.random.default_rng(E * 1000 + N)
    a, b = _lap(E, C, 64), _lap(E, C, 64)
    a.ref_insert_fused, b.ref_insert_fused = False, True
    prio = rng.gamma(0.7, 2.0, (E, C)).astype(np.float32) + np.float32(1e-3)
    for lap in (a, b):
        _set_priorities(lap, prio)
    T = lambda x: torch.as_tensor(x, device="cuda")  # noqa: E731
    strata = (np.arange(N) % E).astype(np.int32)
    for step in range(6):
        st = rng.normal(size=(N, 80)).astype(np.float32)
        nx = rng.normal(size=(N, 80)).astype(np.float32)
        ac = rng.uniform(-1, 1, (N, 7)).astype(np.float32)
        rw = rng.normal(size=N).astype(np.float32)
        dn = rng.random(N) < 0.05
        if step % 2:
            strata = rng.integers(0, E, N).astype(np.int32)
        active = rng.random(N) < [1.0, 0.6, 0.05, 0.95, 0.3, 1.0][step]
        active[rng.integers(0, N - 600):][:500] = False  # a run of done envs
        for lap in (a, b):
            lap.add_batch_ref(T(st), T(ac), T(nx), T(rw), T(dn), T(strata), T(active))
        torch.cuda.synchronize()
        assert a.ref_pointer() == b.ref_pointer(), step
        for name in ("state", "action", "next_state", "reward", "not_done"):
            torch.testing.assert_close(getattr(b, name), getattr(a, name), rtol=0, atol=0)
        torch.testing.assert_close(b._tree, a._tree, rtol=0, atol=0)
        assert torch.equal(a.size_s, b.size_s)
        assert int(b._ref_ws[0]) == 0  # the ticket is left zero
    tr = b._tree.cpu().numpy()
    cap = b._cap
    for s in range(E):
        np.testing.assert_array_equal(tr[s, 1:cap], tr[s, 2:2 * cap:2] + tr[s, 3:2 * cap:2])


def test_fused_ref_insert_with_mask_advance_equals_two_launches():
    """lap_store_batch_ref_fused_adv (the reference-schedule rollout's insert
    with the trainer's mask advance and score accumulation in its last
    workgroup out, r04) against lap_store_batch_ref_fused followed by
    exo_active_advance_score: storage, trees, pointer, mask, step counter,
    count and float64 scores bit for bit, past the table's last row."""
    from exo_amd import _native as nat
    E, C, N, rows = 8, 5000, 4100, 5
    rng = np.random.default_rng(17)
    a, b = _lap(E, C, 64), _lap(E, C, 64)
    a.ref_insert_fused = b.ref_insert_fused = True
    T = lambda x: torch.as_tensor(x, device="cuda")  # noqa: E731
    table = T(rng.random((rows, N)) < 0.8).contiguous()
    strata = T((np.arange(N) % E).astype(np.int32))
    st_a = [table[0].clone(), torch.zeros(1, dtype=torch.int64, device="cuda"),
            torch.zeros(1, dtype=torch.int32, device="cuda"), T(rng.normal(size=N))]
    st_b = [x.clone() for x in st_a]
    for step in range(rows + 2):
        st = T(rng.normal(size=(N, 80)).astype(np.float32))
        nx = T(rng.normal(size=(N, 80)).astype(np.float32))
        ac = T(rng.uniform(-1, 1, (N, 7)).astype(np.float32))
        rw = T(rng.normal(size=N).astype(np.float32))
        dn = T(rng.random(N) < 0.05)
        act_a, k_a, cnt_a, sc_a = st_a
        a.add_batch_ref(st, ac, nx, rw, dn, strata, act_a)
        nat.check(nat.lib().exo_active_advance_score(nat.ptr(table), rows, N, nat.ptr(k_a), nat.ptr(act_a),
                                                     nat.ptr(cnt_a), nat.ptr(rw), nat.ptr(sc_a),
                                                     nat.stream_ptr(torch.device("cuda", 0))), "advance")
        act_b, k_b, cnt_b, sc_b = st_b
        b.add_batch_ref(st, ac, nx, rw, dn, strata, act_b, advance=(table, k_b, cnt_b, sc_b))
        torch.cuda.synchronize()
        assert a.ref_pointer() == b.ref_pointer(), step
        for name in ("state", "action", "next_state", "reward", "not_done"):
            torch.testing.assert_close(getattr(b, name), getattr(a, name), rtol=0, atol=0)
        torch.testing.assert_close(b._tree, a._tree, rtol=0, atol=0)
        for x, y in zip(st_a, st_b):
            assert torch.equal(x, y), step
        assert int(k_b) == min(step + 1, rows - 1)


@pytest.mark.parametrize("C,B,size", [(30_000, 128, 30_000), (30_000, 128, 17_001), (40, 16, 40), (250_000, 64, 99)])
def test_update_and_sample_in_one_launch_equals_two(C, B, size):
    """lap_update_sample_rng (r04): LAP.update_priority then the next sample in
    ONE launch -- the descent reading the top levels the update left in LDS --
    against update_priority() then sample(): every tree node, max_priority,
    the sampled indices and gathered rows, and the RNG call counter, bit for
    bit; non-integer priorities, duplicate update indices, sampling sizes below
    the capacity (the prefix-total path), small and full-depth trees."""
    E = 8
    rng = np.random.default_rng(C + B)
    a, b = _lap(E, C, B), _lap(E, C, B)
    prio = rng.gamma(0.7, 2.0, (E, C)).astype(np.float32) + np.float32(1e-3)
    for lap in (a, b):
        _set_priorities(lap, prio)
        for name in ("state", "action", "next_state", "reward", "not_done"):
            t = getattr(lap, name)
            t.copy_(torch.as_tensor(np.random.default_rng(5).normal(size=t.shape).astype(np.float32)))
        lap.size_s.fill_(size)
    b.fuse_update_sample = True
    for it in range(4):
        idx = rng.integers(0, size, (E, B)).astype(np.int32)
        idx[:, 1::5] = idx[:, ::5][:, :idx[:, 1::5].shape[1]]  # duplicates: the last one wins
        p = torch.as_tensor(rng.uniform(0.1, 9.0, E * B).astype(np.float32), device="cuda")
        ind = torch.as_tensor(idx, device="cuda")
        a.update_priority(p, ind)
        ba = a.sample(it % 2)
        bb = b.update_priority_and_sample(p, ind, it % 2)
        torch.cuda.synchronize()
        torch.testing.assert_close(b._tree, a._tree, rtol=0, atol=0)
        assert float(a._maxp) == float(b._maxp)
        assert torch.equal(a.ind, b.ind)
        for x, y in zip(ba, bb):
            torch.testing.assert_close(y, x, rtol=0, atol=0)
        assert torch.equal(a._rng.state, b._rng.state)


def test_wave_descent_and_subtree_rebuild_match_the_binary_tree():
    """r03d kernels (lap.hip rebuild_subtrees, prefix_total_wave, descend_wave)
    with NON-integer priorities at full depth (2^18 leaves): after batched
    updates with duplicates every internal node is exactly left + right in
    fp32 (the level-by-level recomputation's sums), and the wavefront descent
    of sample() returns exactly the per-thread binary descent of
    sample_indices() -- the same comparisons and subtractions."""
    E, C, B = 3, 250_000, 512
    lap = _lap(E, C, B)
    assert lap._cap == 1 << 18
    rng = np.random.default_rng(7)
    prio = rng.gamma(0.7, 2.0, (E, C)).astype(np.float32) + np.float32(1e-3)
    _set_priorities(lap, prio)
    for _ in range(4):  # random batches with duplicates, like update_priority after a sample
        idx = rng.integers(0, C, (E, B)).astype(np.int32)
        idx[:, 1::7] = idx[:, ::7][:, :idx[:, 1::7].shape[1]]
        p = rng.uniform(0.1, 5.0, (E, B)).astype(np.float32)
        lap.update_priority(torch.as_tensor(p.reshape(-1), device="cuda"),
                            ind=torch.as_tensor(idx, device="cuda"))
    T = lap._tree.cpu().numpy()
    cap = lap._cap
    for s in range(E):
        np.testing.assert_array_equal(T[s, 1:cap], T[s, 2:2 * cap:2] + T[s, 3:2 * cap:2])
    for size in (C, 180_001, 77):
        lap.size_s.fill_(size)
        u = torch.as_tensor(rng.uniform(0, 1, (E, B)).astype(np.float32), device="cuda")
        want = lap.sample_indices(u).cpu().numpy()
        lap.device_rng = False
        lap._u.copy_(u)
        lap._u.uniform_ = lambda: lap._u  # keep the injected uniforms
        lap.sample()
        np.testing.assert_array_equal(lap.ind.cpu().numpy(), want)
        assert want.max() < size


@pytest.mark.parametrize("C", [25_000, 5_000])
def test_store_span_propagation_keeps_the_tree_exact(C):
    """lap_store_rank_kernel (r03d): a stratum's new slots are one ring span
    whose ancestors are recomputed once (propagate_span) -- over several
    4,096-row chunks, ring wrap-around, and (C = 5,000) more rows in one call
    than the ring holds.  Non-integer priorities already in the tree: every
    internal node must be exactly left + right, the new leaves max_priority,
    the others untouched, and ptr / size as the sequential ring."""
    E, n = 3, 20_000
    lap = _lap(E, C, 64)
    rng = np.random.default_rng(11)
    prio = rng.gamma(0.7, 2.0, (E, C)).astype(np.float32) + np.float32(1e-3)
    _set_priorities(lap, prio)
    p0 = lap.max_priority
    want = prio.copy()
    ptr, size = np.zeros(E, np.int64), np.zeros(E, np.int64)
    for step in range(4):
        strata = rng.integers(0, E, n).astype(np.int32)
        active = rng.uniform(size=n) < 0.8
        obs = torch.zeros(n, 80, device="cuda")
        lap.add_batch(obs, torch.zeros(n, 7, device="cuda"), obs, torch.zeros(n, device="cuda"),
                      torch.zeros(n, device="cuda"), torch.as_tensor(strata, device="cuda"),
                      torch.as_tensor(active, device="cuda"))
        for s in range(E):
            k = int(np.sum((strata == s) & active))
            want[s, (ptr[s] + np.arange(k)) % C] = p0
            ptr[s] = (ptr[s] + k) % C
            size[s] = min(size[s] + k, C)
    np.testing.assert_array_equal(lap.ptr_s.cpu().numpy(), ptr)
    np.testing.assert_array_equal(lap.size_s.cpu().numpy(), size)
    np.testing.assert_array_equal(lap.priority.cpu().numpy(), want)
    T = lap._tree.cpu().numpy()
    cap = lap._cap
    for s in range(E):
        np.testing.assert_array_equal(T[s, 1:cap], T[s, 2:2 * cap:2] + T[s, 3:2 * cap:2])


@pytest.mark.parametrize("fused", ["0", "1"])
@pytest.mark.parametrize("n,cap,steps", [(4096, 30000, 5), (1000, 2048, 9), (8192, 9000, 3)])
def test_vectorised_insert_equals_per_row_ring_adds(n, cap, steps, fused, monkeypatch):
    """lap_store_batch (r05: one launch up to 8,192 rows -- scan, leaves, span
    propagation and the row copies in one workgroup per stratum) against the
    per-stratum ring semantics row by row: rows of stratum s in env order to
    slots ptr_s, ptr_s + 1, ... (mod capacity), leaves = max_priority, every
    inner node the sum of its children; random masks and strata, ring wraps
    across calls.  fused: the opt-in one-launch insert (EXO_LAP_STORE_FUSED=1,
    measured slower in the loop) against the same semantics."""
    monkeypatch.setenv("EXO_LAP_STORE_FUSED", fused)
    E = 8
    lap = _lap(E, cap, 16)
    g = torch.Generator(device="cuda").manual_seed(n + cap)
    strata = torch.randint(0, E, (n,), device="cuda", generator=g, dtype=torch.int32)
    ptr = np.zeros(E, dtype=np.int64)
    size = np.zeros(E, dtype=np.int64)
    want_state = np.zeros((E, cap + 1), dtype=np.float32)
    st_h = strata.cpu().numpy()
    for k in range(steps):
        active = torch.rand(n, device="cuda", generator=g) < 0.8
        obs = torch.randn(n, 80, device="cuda", generator=g)
        nobs = torch.randn(n, 80, device="cuda", generator=g)
        act = torch.rand(n, 7, device="cuda", generator=g) * 2 - 1
        rew = torch.randn(n, device="cuda", generator=g)
        done = torch.rand(n, device="cuda", generator=g) < 0.1
        lap.add_batch(obs, act, nobs, rew, done, strata, active)
        a_h, o_h = active.cpu().numpy(), obs[:, 0].cpu().numpy()
        for i in range(n):
            if a_h[i]:
                s = st_h[i]
                want_state[s, ptr[s]] = o_h[i]
                ptr[s] = (ptr[s] + 1) % cap
                size[s] = min(size[s] + 1, cap)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(lap.ptr_s.cpu().numpy(), ptr)
    np.testing.assert_array_equal(lap.size_s.cpu().numpy(), size)
    np.testing.assert_array_equal(lap.state[:, :cap, 0].cpu().numpy(), want_state[:, :cap])
    tree = lap._tree.cpu().numpy().astype(np.float64)
    c2 = tree.shape[1] // 2
    for s in range(E):
        leaves = tree[s, c2:]
        assert np.all(leaves[:size[s]] == 1.0) and np.all(leaves[size[s]:cap] == 0.0)
        assert tree[s, 1] == float(size[s])  # integer sums: exact at any order


@pytest.mark.parametrize("E,C,n,rows,p_act", [(8, 40, 37, 9, 0.5), (8, 4096, 300, 12, 0.9), (4, 23, 11, 7, 0.15),
                                             (8, 5000, 4096, 4, 0.97)])
def test_planned_round_equals_per_step_reference_inserts(E, C, n, rows, p_act):
    """lap_ref_plan + lap_ref_step per row + lap_ref_commit (the reference
    schedule's planned rollout inserts, r05) against add_batch_ref per row (the
    per-step inserts, pinned to the sequential adds above): storage, every tree
    node, pointer and sizes bit for bit after every round, and every internal
    node exactly left + right.  Rounds cover the last add landing one slot past
    ptr0 + adv - 1 (count0 + total - 1 not a multiple of E), a
    round with fewer adds than E, an empty round and a ring that wraps."""
    rng = np.random.default_rng(C + n)
    a, b = _lap(E, C, 16), _lap(E, C, 16)
    T = lambda x: torch.as_tensor(x, device="cuda")  # noqa: E731
    strata = T(rng.integers(0, E, n).astype(np.int32))
    kk = torch.zeros((2,), dtype=torch.int64, device="cuda")
    wrapped = False
    for rnd in range(8):
        p = [p_act, 2.0 / (n * rows), 0.0, p_act, 0.6, p_act, 1.0, 0.3][rnd]
        table = rng.random((rows, n)) < p
        if rnd == 1:
            table[:] = False
            table[rows // 2, : max(1, E // 2 - 1)] = True  # fewer adds than strata
        if rnd == 5:  # a max_priority other than 1 for this round's leaves
            pr = torch.full((E * 16,), 2.5 + rnd, device="cuda")
            for lap in (a, b):
                lap.update_priority(pr, ind=torch.zeros((E, 16), dtype=torch.int32, device="cuda"))
        tb = T(table.astype(np.uint8))
        counts = tb.sum(1).to(torch.int64)
        offs, total = torch.cumsum(counts, 0) - counts, int(counts.sum())
        plan = torch.full((rows, n), -1, dtype=torch.int32, device="cuda")
        kk.zero_()
        b.ref_plan(tb, strata, offs, total, plan)
        active_b = tb[0].clone()
        for k in range(rows):
            st, nx = T(rng.normal(size=(n, 80)).astype(np.float32)), T(rng.normal(size=(n, 80)).astype(np.float32))
            ac = T(rng.uniform(-1, 1, (n, 7)).astype(np.float32))
            rw, dn = T(rng.normal(size=n).astype(np.float32)), T(rng.random(n) < 0.1)
            a.add_batch_ref(st, ac, nx, rw, dn, strata, tb[k])
            b.ref_step(plan, tb, kk, k % 2, st, ac, nx, rw, dn, strata, active_b)
        b.ref_commit(plan, strata, total)
        torch.cuda.synchronize()
        ptr, count, _ = a.ref_pointer()
        assert b.ref_pointer() == a.ref_pointer(), rnd
        wrapped |= count > C
        for name in ("state", "action", "next_state", "reward", "not_done"):
            torch.testing.assert_close(getattr(b, name)[:, :C], getattr(a, name)[:, :C], rtol=0, atol=0,
                                       msg=f"{name} round {rnd}")
        torch.testing.assert_close(b._tree, a._tree, rtol=0, atol=0, msg=f"tree round {rnd}")
        assert torch.equal(a.size_s, b.size_s)
        tr, cap = b._tree.cpu().numpy(), b._cap
        for s in range(E):
            np.testing.assert_array_equal(tr[s, 1:cap], tr[s, 2:2 * cap:2] + tr[s, 3:2 * cap:2])
    assert wrapped or C >= 4096


def test_lap_rejects_trees_deeper_than_the_prefix_walk():
    """prefix_sum unrolls 24 levels: a stratum capacity above 2^24 is refused
     instead of sampling against a truncated prefix total."""
    from exo_amd.replay import LAP
    with pytest.raises(ValueError):
        LAP(80, 7, "cuda", 1, max_size=(1 << 24) + 1, batch_size=4)
