"""Data-parallel TD7 at the bench's widths on the GPU: two
gloo ranks, both on cuda:0 (a one-GPU box), each fed one half of an injected
8 x 128 batch (tests/helpers.td7_full_batch, with its target-policy noise),
must end where ONE process lands that trains on the whole batch -- the
reference's update on the full batch (Agent/TD7_multi_agent.py:211-293): every
loss is a batch mean, so the average of the two half-batch gradients is the
full-batch gradient up to fp32 summation order.  Three updates, the second
with the actor step, then a target refresh (MAX-reduced Q bounds).
The two replicas must be bit-identical.

Tolerances: fp32 (exact f32 MFMA) as tests/test_dp_gloo.py, rtol 2e-5 /
atol 2e-6 on the parameters; bf16 (the bench's fused kernels) 1e-4 / 1e-5 --
the operands are rounded to bf16 identically on both sides (row-local
forward), so only the weight-gradient reduction order over the batch differs,
amplified by at most Adam's per-element normalisation of the first steps.  A
parameter whose gradient sits at the rounding noise can flip the sign of an
early Adam update (a step of ~2 lr); such entries may number at most 1e-3 of
all and move by at most 2 lr per update."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu
STEPS = 3
TOL = {"fp32": (2e-5, 2e-6), "bf16": (1e-4, 1e-5)}


def _port():
    from _ports import free_port
    return free_port()


def _learner(precision, sync=None, seed=0):
    from exo_amd.td7 import GradSync, Hyperparameters, TD7Learner
    from helpers import TD7_FULL_HP
    torch.manual_seed(seed)
    hp = Hyperparameters(**dict(TD7_FULL_HP, target_update_rate=STEPS))
    return TD7Learner(80, 7, hp, device="cuda:0", precision=precision, sync=sync or GradSync(None))


def _train(L, part):
    from helpers import td7_full_batch
    for step in range(STEPS):
        b = [torch.as_tensor(x, device="cuda:0") for x in td7_full_batch(step)]
        if part is not None:
            rank, world = part
            n = b[0].shape[0] // world
            b = [x[rank * n:(rank + 1) * n].contiguous() for x in b]
        L.update(*b[:5], noise=b[5])
        L.maybe_update_targets()
    torch.cuda.synchronize()
    out = {f"{n}.{k}": v.detach().cpu().clone() for n in ("actor", "critic", "encoder", "fixed_encoder", "critic_target")
           for k, v in getattr(L, n).state_dict().items()}
    out["max"], out["min"] = L.max.cpu().clone(), L.min.cpu().clone()
    return out


def _worker(rank, world, port, outdir, precision):
    sys.path.insert(0, HERE)
    import conftest  # noqa: F401  (sys.path)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from exo_amd.td7 import GradSync
    L = _learner(precision, GradSync(dist.group.WORLD), seed=100 + rank)  # rank 0's init is broadcast
    torch.save(_train(L, (rank, world)), os.path.join(outdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_two_ranks_on_halves_match_one_rank_on_the_batch(tmp_path, precision):
    world = 2
    mp.spawn(_worker, args=(world, _port(), str(tmp_path), precision), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for k in r0:
        torch.testing.assert_close(r0[k], r1[k], rtol=0, atol=0, msg=f"replicas differ: {k}")
    single = _train(_learner(precision, seed=100), None)
    rtol, atol = TOL[precision]
    outliers = total = 0
    for k, v in single.items():
        a, b = r0[k].double().numpy(), v.double().numpy()
        bad = np.abs(a - b) > atol + rtol * np.abs(b)
        total += a.size
        if k in ("max", "min"):
            assert not bad.any(), f"{k}: {a} vs {b}"
            continue
        outliers += int(bad.sum())
        # an Adam step is at most ~lr per update: a sign-flipped early step of a
        # noise-level gradient moves an entry by a few lr, never more
        assert not bad.any() or np.abs(a - b)[bad].max() <= 2 * 3e-4 * STEPS, \
            f"{k}: max |dp - single| {np.abs(a - b)[bad].max():.3g}"
    assert outliers <= 1e-3 * total, f"{outliers} of {total} entries outside rtol {rtol} / atol {atol}"
