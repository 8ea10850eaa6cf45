"""Per-launch time of FlatAdam.step_many (encoder + critic, one
td7_adam_step_multi launch) vs the flat single-optimiser td7_adam_step, graph
replayed (tools/dense_bench.py timing), and the bytes each moves."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dense_bench import timeit  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from exo_amd.td7 import Critic, Encoder, FlatAdam  # noqa: E402


def main():
    torch.manual_seed(0)
    nets = [Encoder(80, 7, 300, 300, F.elu).cuda(), Critic(80, 7, 300, 320, F.elu).cuda()]
    opts = [FlatAdam(n, lr=3e-4, weight_decay=1e-7) for n in nets]
    for n in nets:
        for p in n.parameters():
            p.grad = torch.randn_like(p) * 1e-3
    FlatAdam.step_many(opts)
    n_par = sum(o.flat.numel() for o in opts)
    t_multi = timeit(lambda: FlatAdam.step_many(opts))
    flat = torch.randn(opts[1].flat.numel(), device="cuda") * 1e-3
    t_flat = timeit(lambda: opts[1].step(flat_grad=flat))
    gb = n_par * 4 * 7 / 1e9
    print(f"step_many over {n_par} params: {t_multi:.2f} us ({gb / (t_multi * 1e-6):.0f} GB/s); "
          f"single flat step over {opts[1].flat.numel()}: {t_flat:.2f} us")


if __name__ == "__main__":
    main()
