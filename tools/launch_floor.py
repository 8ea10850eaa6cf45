"""Per-kernel cost of back-to-back small torch kernels replayed from a HIP
graph (the TD7 update is ~300 of them): wall time per replay / kernels."""
import time

import torch


def bench(n_kernels=200, shape=(1024, 300), reps=50):
    x = torch.randn(*shape, device="cuda")
    y = torch.randn(*shape, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n_kernels):
                x.add_(y)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps / n_kernels * 1e6
    print(f"{shape} add_: {dt:.2f} us per kernel in a graph", flush=True)


if __name__ == "__main__":
    for shp in ((1024, 300), (64,), (4096, 300), (1024, 1200)):
        bench(shape=shp)
