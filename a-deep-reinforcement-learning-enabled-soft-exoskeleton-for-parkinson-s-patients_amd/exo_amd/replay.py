"""LAP prioritised replay on the GPU (reference: Agent/TD7_buffer_multi_agent.py).

Storage is fp32 on the device ([strata, max_size + 1, dim]; the extra row per
stratum absorbs writes of inactive envs so batched inserts need no host sync),
priorities are per-stratum sum trees updated and sampled by the HIP kernels in
csrc/lap.hip.  The reference stores float64 numpy arrays and converts every
sampled batch to float32 on the way to the device (:105-111); storing float32
gives the same training inputs.

Two insert paths:
* add(...)       -- one transition, the reference's exact pointer semantics
                    (ptr advances when count % num_envs == 0 BEFORE count is
                    incremented, :59-63);
* add_batch(...) -- one vectorised env step: a ring per stratum, one slot per
                    active env-step (documented divergence);
* add_batch_ref(...) -- one vectorised env step as the training script's
                    per-env add loop (Exoskeleton_agent_train.py:139-142): the
                    reference's shared pointer, kept on the device
                    (lap_store_batch_ref), so a vectorised run fills the buffer
                    slot for slot like the script's sequential adds.
"""
import ctypes
import os

import numpy as np
import torch

from . import _native as nat


class LAP:
    def __init__(self, state_dim, action_dim, device, num_envs, max_size=1e6, batch_size=64, max_action=1,
                 normalize_actions=True, prioritized=True):
        if not prioritized:
            raise NotImplementedError("only the prioritized LAP buffer of the TD7 agent is implemented")
        self.device = nat.require_gpu(device)
        self.max_size = int(max_size)
        self.max_action = max_action
        self.batch_size = int(batch_size)
        self.num_envs = int(num_envs)
        self.state_dim, self.action_dim = state_dim, action_dim
        self.normalize_actions = max_action if normalize_actions else 1
        self.prioritized = True
        E, C = self.num_envs, self.max_size
        if C > 1 << 24:  # csrc/lap.hip prefix_sum walks at most 24 levels
            raise ValueError(f"LAP: max_size {C} above 2^24 rows per stratum")
        f32 = dict(device=self.device, dtype=torch.float32)
        self.state = torch.zeros((E, C + 1, state_dim), **f32)
        self.action = torch.zeros((E, C + 1, action_dim), **f32)
        self.next_state = torch.zeros((E, C + 1, state_dim), **f32)
        self.reward = torch.zeros((E, C + 1, 1), **f32)
        self.not_done = torch.zeros((E, C + 1, 1), **f32)
        cap = 1
        while cap < C:
            cap <<= 1
        self._tree = torch.zeros((E, 2 * cap), **f32)
        self._maxp = torch.ones((1,), **f32)
        self._desc = nat.LapTreeDesc(self._tree.data_ptr(), self._maxp.data_ptr(), E, C, cap)
        self._cap = cap
        # reference pointer semantics (single add)
        self.ptr = 0
        self.count = 0
        self.size = 0
        # per-stratum rings (batched add), device-resident
        i32 = dict(device=self.device, dtype=torch.int32)
        self.ptr_s = torch.zeros((E,), **i32)
        self.size_s = torch.zeros((E,), **i32)
        self._row0 = (torch.arange(E, device=self.device, dtype=torch.int64) * (C + 1))
        self.ind = None
        # reference pointer of add_batch_ref: int64 {ptr, count, size} on the device
        self.ref_state = torch.zeros((3,), dtype=torch.int64, device=self.device)
        self._ref_ws = None
        self.ref_insert_fused = os.environ.get("EXO_REF_INSERT_FUSED", "1") != "0"
        self._u = torch.empty((E, self.batch_size), **f32)
        # sample() draws its uniforms in the kernel (EXO_DEVICE_RNG=0: torch.rand + lap_sample_gather)
        from .ops import DeviceRNG
        self.device_rng = os.environ.get("EXO_DEVICE_RNG", "1") != "0"
        self._rng = DeviceRNG(self.device, 3)
        self._idx = torch.empty((E, self.batch_size), **i32)
        self._store = nat.LapStorageDesc(self.state.data_ptr(), self.action.data_ptr(), self.next_state.data_ptr(),
                                         self.reward.data_ptr(), self.not_done.data_ptr(), state_dim, action_dim,
                                         self.ptr_s.data_ptr(), self.size_s.data_ptr())
        B = E * self.batch_size  # sampled batch, written in place by lap_sample_gather (static for HIP graphs)
        # state and next_state adjacent in one [2, B, dim] buffer: the learner's
        # paired passes over both read it as one tensor (ops.pair_rows), no stack / cat
        sn = torch.empty((2, B, state_dim), **f32)
        self._batch = (sn[0], torch.empty((B, action_dim), **f32), sn[1], torch.empty((B, 1), **f32),
                       torch.empty((B, 1), **f32))
        self._row_ws = None
        self._init_tree()

    def _stream(self):
        return nat.stream_ptr(self.device)

    def _init_tree(self):
        nat.check(nat.lib().lap_init(ctypes.byref(self._desc), self._stream()), "lap_init")

    # --------------------------------------------------------------- views
    @property
    def priority(self):
        """[E, max_size] view of the tree leaves (the reference's self.priority)."""
        return self._tree[:, self._cap:self._cap + self.max_size]

    @property
    def max_priority(self):
        return float(self._maxp)

    @property
    def totals(self):
        return self._tree[:, 1]

    # ---------------------------------------------------------------- adds
    def add(self, state, action, next_state, reward, done, tremor_num):
        """Agent/TD7_buffer_multi_agent.py:49-63."""
        s, p = int(tremor_num), self.ptr
        dev = self.device
        self.state[s, p] = torch.as_tensor(np.asarray(state, dtype=np.float32), device=dev)
        self.action[s, p] = torch.as_tensor(np.asarray(action, dtype=np.float32) / self.normalize_actions, device=dev)
        self.next_state[s, p] = torch.as_tensor(np.asarray(next_state, dtype=np.float32), device=dev)
        self.reward[s, p] = float(reward)
        self.not_done[s, p] = 1.0 - float(done)
        st = torch.tensor([s], dtype=torch.int32, device=dev)
        sl = torch.tensor([p], dtype=torch.int32, device=dev)
        nat.check(nat.lib().lap_add(ctypes.byref(self._desc), nat.ptr(st), nat.ptr(sl), 1, self._stream()), "lap_add")
        if self.count % self.num_envs == 0:
            self.ptr = (self.ptr + 1) % self.max_size
            self.size = min(self.size + 1, self.max_size)
        self.count += 1
        self.size_s.fill_(self.size)

    def add_batch(self, state, action, next_state, reward, done, strata, active=None):
        """One vectorised env step: row i goes to stratum strata[i] (int32 [N]) if
        active[i] (bool/uint8 [N], default all) -- lap_store_batch, two kernels,
        no host synchronisation."""
        n = state.shape[0]
        if self._row_ws is None or self._row_ws.numel() < n:
            self._row_ws = torch.empty((n,), dtype=torch.int32, device=self.device)

        def f32(t, shape):
            t = t.to(device=self.device, dtype=torch.float32).reshape(shape)
            return t if t.is_contiguous() else t.contiguous()

        st = f32(state, (n, self.state_dim))
        nx = f32(next_state, (n, self.state_dim))
        ac = f32(action, (n, self.action_dim))
        rw = f32(reward, (n,))
        dn = done if done.dtype == torch.uint8 else (done.view(torch.uint8) if done.dtype == torch.bool
                                                     else done.to(torch.uint8))
        dn = dn.reshape(n).contiguous()
        sr = strata if strata.dtype == torch.int32 else strata.to(torch.int32)
        act = None
        if active is not None:
            act = active.view(torch.uint8) if active.dtype == torch.bool else active.to(torch.uint8)
            act = act.contiguous()
        nat.check(nat.lib().lap_store_batch(ctypes.byref(self._desc), ctypes.byref(self._store), nat.ptr(st),
                                            nat.ptr(ac), nat.ptr(nx), nat.ptr(rw), nat.ptr(dn), nat.ptr(sr.contiguous()),
                                            nat.ptr(act), float(self.normalize_actions), n, nat.ptr(self._row_ws),
                                            self._stream()), "lap_store_batch")

    def add_batch_ref(self, state, action, next_state, reward, done, strata, active=None, advance=None):
        """LAP.add (:49-63) for every active row in row order -- the training
        script's per-env loop over one vectorised step -- with the reference's
        shared pointer (ref_state, device-resident): env 0's first transition
        one slot behind the others, a done env's slot re-used by the next adds,
        one shared sampling size.  One kernel (lap_store_batch_ref_fused, r04;
        EXO_REF_INSERT_FUSED=0: the three launches of lap_store_batch_ref), no
        host synchronisation.  advance = (table, k, count, score): the
        trainer's mask advance in the same launch (lap_store_batch_ref_fused_adv;
        `active` is then advanced in place, the rewards added into score)."""
        n = state.shape[0]
        if self._ref_ws is None or self._ref_ws.numel() < 3 * n:
            # zeroed: its first word is the fused launch's ticket (left zero)
            self._ref_ws = torch.zeros((3 * n,), dtype=torch.int32, device=self.device)

        def f32(t, shape):
            t = t.to(device=self.device, dtype=torch.float32).reshape(shape)
            return t if t.is_contiguous() else t.contiguous()

        st = f32(state, (n, self.state_dim))
        nx = f32(next_state, (n, self.state_dim))
        ac = f32(action, (n, self.action_dim))
        rw = f32(reward, (n,))
        dn = done if done.dtype == torch.uint8 else (done.view(torch.uint8) if done.dtype == torch.bool
                                                     else done.to(torch.uint8))
        dn = dn.reshape(n).contiguous()
        sr = (strata if strata.dtype == torch.int32 else strata.to(torch.int32)).contiguous()
        act = None
        if active is not None:
            act = (active.view(torch.uint8) if active.dtype == torch.bool else active.to(torch.uint8)).contiguous()
        if advance is not None:
            if not self.ref_insert_fused or act is None or act.data_ptr() != active.data_ptr():
                raise ValueError("add_batch_ref(advance=...): the fused insert and an in-place uint8/bool mask only")
            table, k, count, score = advance
            nat.check(nat.lib().lap_store_batch_ref_fused_adv(
                ctypes.byref(self._desc), ctypes.byref(self._store), nat.ptr(self.ref_state), nat.ptr(st),
                nat.ptr(ac), nat.ptr(nx), nat.ptr(rw), nat.ptr(dn), nat.ptr(sr), nat.ptr(act),
                float(self.normalize_actions), n, nat.ptr(self._ref_ws), nat.ptr(table), table.shape[0], nat.ptr(k),
                nat.ptr(count), nat.ptr(score), self._stream()), "lap_store_batch_ref_fused_adv")
            return
        fn = "lap_store_batch_ref_fused" if self.ref_insert_fused else "lap_store_batch_ref"
        nat.check(getattr(nat.lib(), fn)(ctypes.byref(self._desc), ctypes.byref(self._store),
                                         nat.ptr(self.ref_state), nat.ptr(st), nat.ptr(ac), nat.ptr(nx),
                                         nat.ptr(rw), nat.ptr(dn), nat.ptr(sr), nat.ptr(act),
                                         float(self.normalize_actions), n, nat.ptr(self._ref_ws),
                                         self._stream()), fn)

    # ----------------------------------------------- planned reference inserts
    # (lap_ref_plan / lap_ref_step / lap_ref_commit, csrc/lap.hip): a whole
    # synchronous episode round of add_batch_ref calls planned at its start --
    # the steps' envs come from a fixed mask table -- so a step is one
    # elementwise launch and the tree is updated once, at ref_commit.  Bit
    # for bit the per-step inserts' rows, leaves, sums, pointer and sizes,
    # provided nothing reads the tree between ref_plan and ref_commit.
    def ref_plan(self, table, strata, offs, total, plan):
        """plan[k][e] (int32 [rows][n]) for the mask table rows (uint8/bool
        [rows][n]); offs: int64 device [rows], the adds before each row."""
        rows, n = table.shape
        if getattr(self, "_ref_add_ws", None) is None or self._ref_add_ws.numel() < max(int(total), 1):
            self._ref_add_ws = torch.empty((max(int(total), 1),), dtype=torch.int32, device=self.device)
        tb = table.view(torch.uint8) if table.dtype == torch.bool else table
        sr = (strata if strata.dtype == torch.int32 else strata.to(torch.int32)).contiguous()
        nat.check(nat.lib().lap_ref_plan(ctypes.byref(self._desc), nat.ptr(self.ref_state), nat.ptr(tb), rows, n,
                                         nat.ptr(sr), nat.ptr(offs), int(total), nat.ptr(self._ref_add_ws),
                                         nat.ptr(plan), self._stream()), "lap_ref_plan")

    def ref_step(self, plan, table, kk, par, state, action, next_state, reward, done, strata, active,
                 k_dev=None, count=None, counts_table=None, score=None):
        """One step of a planned round (see ref_plan): the transitions to their
        planned slots, score += reward where active, the next mask in place."""
        rows, n = plan.shape
        tb = table.view(torch.uint8) if table.dtype == torch.bool else table
        dn = done.view(torch.uint8) if done.dtype == torch.bool else done.to(torch.uint8)
        act = active.view(torch.uint8) if active.dtype == torch.bool else active
        nat.check(nat.lib().lap_ref_step(
            ctypes.byref(self._desc), ctypes.byref(self._store), nat.ptr(plan), rows, n, nat.ptr(kk), int(par),
            nat.ptr(k_dev), nat.ptr(strata), nat.ptr(state.contiguous()), nat.ptr(action.contiguous()),
            nat.ptr(next_state.contiguous()), nat.ptr(reward.contiguous()), nat.ptr(dn.contiguous()),
            float(self.normalize_actions), nat.ptr(tb), nat.ptr(act), nat.ptr(count), nat.ptr(counts_table),
            nat.ptr(score), self._stream()), "lap_ref_step")

    def ref_commit(self, plan, strata, total):
        """The end of a planned round: leaves, the round's span, the pointer."""
        rows, n = plan.shape
        nat.check(nat.lib().lap_ref_commit(ctypes.byref(self._desc), ctypes.byref(self._store),
                                           nat.ptr(self.ref_state), nat.ptr(plan), rows, n, nat.ptr(strata),
                                           int(total), self._stream()), "lap_ref_commit")

    def ref_pointer(self):
        """(ptr, count, size) of add_batch_ref (host sync)."""
        return tuple(int(v) for v in self.ref_state.cpu())

    # ------------------------------------------------------------- sample
    def _slot(self, slot):
        """Batch buffers of sample(slot=...): the vectorised trainer samples the
        next iteration's batch into the other slot while this one is in use."""
        if slot is None:
            return self._batch, self._idx
        if not hasattr(self, "_slots"):
            self._slots = {}
        if slot not in self._slots:
            f32 = dict(device=self.device, dtype=torch.float32)
            B, (S, A) = self._batch[0].shape[0], (self._batch[0].shape[1], self._batch[1].shape[1])
            sn = torch.empty((2, B, S), **f32)
            self._slots[slot] = ((sn[0], torch.empty((B, A), **f32), sn[1], torch.empty((B, 1), **f32),
                                  torch.empty((B, 1), **f32)), torch.empty_like(self._idx))
        return self._slots[slot]

    def sample(self, slot=None):
        """Agent/TD7_buffer_multi_agent.py:65-111: batch_size rows from every
        stratum, stratum-major, as float32 device tensors (lap_sample_gather:
        descent + gather in one kernel; the returned tensors are reused by the
        next call with the same slot).  self.ind = the sampled indices."""
        batch, idx = self._slot(slot)
        if self.device_rng:
            # the uniforms drawn inside the kernel (ops.DeviceRNG): no generator launch
            r = self._rng
            nat.check(nat.lib().lap_sample_gather_rng(ctypes.byref(self._desc), ctypes.byref(self._store), r.seed,
                                                      r.tag, r.counter_ptr, r.ticket_ptr, self.batch_size,
                                                      nat.ptr(idx), *[nat.ptr(t) for t in batch],
                                                      self._stream()), "lap_sample_gather_rng")
        else:
            self._u.uniform_()
            nat.check(nat.lib().lap_sample_gather(ctypes.byref(self._desc), ctypes.byref(self._store),
                                                  nat.ptr(self._u), self.batch_size, nat.ptr(idx),
                                                  *[nat.ptr(t) for t in batch], self._stream()),
                      "lap_sample_gather")
        self.ind = idx
        return batch

    def sample_indices(self, u):
        """Indices for given uniforms u [E, batch] (parity hook)."""
        u = u.to(device=self.device, dtype=torch.float32).contiguous()
        idx = torch.empty(u.shape, dtype=torch.int32, device=self.device)
        nat.check(nat.lib().lap_sample(ctypes.byref(self._desc), nat.ptr(u), nat.ptr(self.size_s), u.shape[1],
                                       nat.ptr(idx), self._stream()), "lap_sample")
        return idx

    def update_priority(self, priority, ind=None):
        """:113-117 (max_priority stays on the device)."""
        ind = self.ind if ind is None else ind
        pr = priority.detach().to(torch.float32).reshape(-1).contiguous()
        assert pr.numel() == ind.numel()
        nat.check(nat.lib().lap_update(ctypes.byref(self._desc), nat.ptr(ind), nat.ptr(pr), ind.shape[1],
                                       self._stream()), "lap_update")

    # LAP.update_priority + the next sample as one launch (lap_update_sample_rng,
    # r04); EXO_LAP_FUSED=0: the two launches
    fuse_update_sample = os.environ.get("EXO_LAP_FUSED", "1") != "0"

    def update_priority_and_sample(self, priority, ind=None, slot=None, before_gather=None):
        """update_priority(priority, ind) then sample(slot), the same values; one
        launch with the device RNG (the sampled batch in the slot's buffers,
        self.ind = its indices).  before_gather (a callable, r05): two launches
        instead -- the update and the indices, then before_gather() (the caller's
        stream waits), then the rows gathered (lap_update_sample_idx +
        lap_gather_rows, bit-identical)."""
        ind = self.ind if ind is None else ind
        if not (self.device_rng and self.fuse_update_sample and self.batch_size <= 1024):
            self.update_priority(priority, ind)
            if before_gather is not None:
                before_gather()
            return self.sample(slot)
        pr = priority.detach().to(torch.float32).reshape(-1).contiguous()
        assert pr.numel() == ind.numel()
        batch, idx = self._slot(slot)
        r = self._rng
        if before_gather is not None:
            nat.check(nat.lib().lap_update_sample_idx(ctypes.byref(self._desc), ctypes.byref(self._store), nat.ptr(ind),
                                                      nat.ptr(pr), ind.shape[1], r.seed, r.tag, r.counter_ptr,
                                                      r.ticket_ptr, nat.ptr(idx), self._stream()),
                      "lap_update_sample_idx")
            before_gather()
            nat.check(nat.lib().lap_gather_rows(ctypes.byref(self._desc), ctypes.byref(self._store), ind.shape[1],
                                                nat.ptr(idx), *[nat.ptr(t) for t in batch], self._stream()),
                      "lap_gather_rows")
            self.ind = idx
            return batch
        nat.check(nat.lib().lap_update_sample_rng(ctypes.byref(self._desc), ctypes.byref(self._store), nat.ptr(ind),
                                                  nat.ptr(pr), ind.shape[1], r.seed, r.tag, r.counter_ptr,
                                                  r.ticket_ptr, nat.ptr(idx), *[nat.ptr(t) for t in batch],
                                                  self._stream()), "lap_update_sample_rng")
        self.ind = idx
        return batch

    def update_priority_and_sample_td(self, td, alpha, min_priority, ind, slot, prio_out=None):
        """update_priority_and_sample with the priorities computed in the launch
        from the critic pass's |td| [B, 2] (lap_update_sample_td): the same
        values as td7f_wgrad's, so the update needs only the critic pass."""
        if not (self.device_rng and self.batch_size <= 1024):
            raise RuntimeError("update_priority_and_sample_td: the device RNG and batch <= 1024 only")
        batch, idx = self._slot(slot)
        r = self._rng
        nat.check(nat.lib().lap_update_sample_td(ctypes.byref(self._desc), ctypes.byref(self._store), nat.ptr(ind),
                                                 nat.ptr(td), float(alpha), float(min_priority), nat.ptr(prio_out),
                                                 ind.shape[1], r.seed, r.tag, r.counter_ptr, r.ticket_ptr,
                                                 nat.ptr(idx), *[nat.ptr(t) for t in batch], self._stream()),
                  "lap_update_sample_td")
        self.ind = idx
        return batch

    def reset_max_priority(self):
        nat.check(nat.lib().lap_reset_max(ctypes.byref(self._desc), self._stream()), "lap_reset_max")

    def reset_buffer(self):
        """:122-139"""
        self.ptr = self.count = self.size = 0
        for t in (self.state, self.action, self.next_state, self.reward, self.not_done):
            t.zero_()
        self.ptr_s.zero_()
        self.size_s.zero_()
        self.ref_state.zero_()
        self._init_tree()
