"""Data-parallel TD7 (exo_amd.td7.GradSync) with world_size 2 over gloo on CPU:
ranks that see different halves of a batch must end bit-close to one process
that sees the whole batch, and stay identical to each other."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    from _ports import free_port
    return free_port()


def _hp():
    from exo_amd.td7 import Hyperparameters
    return Hyperparameters(zs_dim=16, enc_hdim=24, critic_hdim=20, actor_hdim=18, batch_size=8)


def _batches(seed, n):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        out.append((torch.randn(16, 80, generator=g), torch.rand(16, 7, generator=g) * 2 - 1,
                    torch.randn(16, 80, generator=g), torch.rand(16, 1, generator=g),
                    (torch.rand(16, 1, generator=g) > 0.1).float(), torch.randn(16, 7, generator=g)))
    return out


def _worker(rank, world, port, outdir):
    sys.path.insert(0, HERE)
    import conftest  # noqa: F401  (sys.path)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from exo_amd.td7 import GradSync, TD7Learner
    torch.manual_seed(100 + rank)  # different init on purpose: rank 0's weights are broadcast
    L = TD7Learner(80, 7, _hp(), device="cpu", sync=GradSync(dist.group.WORLD), fused_adam=False)
    for b in _batches(0, 4):
        half = [x[rank * 8:(rank + 1) * 8] for x in b]
        L.update(*half[:5], noise=half[5])
        L.maybe_update_targets()
    L.sync_bounds()
    sd = {f"{n}.{k}": v.detach().clone() for n in ("actor", "critic", "encoder")
          for k, v in getattr(L, n).state_dict().items()}
    sd["max"] = L.max.clone()
    sd["min"] = L.min.clone()
    torch.save(sd, os.path.join(outdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def test_data_parallel_matches_single_process(tmp_path):
    world, port = 2, _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for k in r0:
        torch.testing.assert_close(r0[k], r1[k], rtol=0, atol=0)
    from exo_amd.td7 import TD7Learner
    torch.manual_seed(100)
    S = TD7Learner(80, 7, _hp(), device="cpu", fused_adam=False)
    for b in _batches(0, 4):
        S.update(*b[:5], noise=b[5])
        S.maybe_update_targets()
    for n in ("actor", "critic", "encoder"):
        for k, v in getattr(S, n).state_dict().items():
            np.testing.assert_allclose(r0[f"{n}.{k}"].numpy(), v.numpy(), rtol=2e-5, atol=2e-6, err_msg=f"{n}.{k}")
    assert float(r0["max"]) == float(S.max) and float(r0["min"]) == float(S.min)


def _forced_worker(rank, world, port, outdir):
    sys.path.insert(0, HERE)
    import helpers  # noqa: F401  (puts the package on sys.path)
    os.environ["EXO_FORCE_DIST"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from exo_amd.td7 import GradSync
    s = GradSync(dist.group.WORLD)
    flat = torch.arange(6, dtype=torch.float32)
    s.allreduce_flat(flat)  # one rank: SUM is the identity
    t = torch.tensor([3.0])
    s.max_(t)
    torch.save({"active": s.active, "world": s.world, "flat": flat, "t": t,
                "plain": GradSync(None).active}, os.path.join(outdir, "forced.pt"))
    dist.destroy_process_group()


def test_force_dist_activates_the_collectives_at_world_one(tmp_path):
    """EXO_FORCE_DIST=1 (bench.py under torchrun with one rank): GradSync is
    active with a process group of one, so the data-parallel layout and its
    collectives run; without a group it stays inactive."""
    mp.spawn(_forced_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    r = torch.load(os.path.join(tmp_path, "forced.pt"), weights_only=True)
    assert r["active"] is True and r["world"] == 1 and r["plain"] is False
    assert torch.equal(r["flat"], torch.arange(6, dtype=torch.float32)) and float(r["t"]) == 3.0
