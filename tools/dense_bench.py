"""Per-launch time of the td7_dense kernels vs torch (hipBLASLt + elementwise)
at the TD7 layer shapes; HIP events around 50 back-to-back launches."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402
from exo_amd import _native as nat  # noqa: E402

# MFMA operand precision (DB_PREC=fp32|bf16|fp16): bits 8-15 of the act code
PREC = {"fp32": 0, "bf16": 1, "fp16": 2}[os.environ.get("DB_PREC", "fp32")]
ACT = 2 | PREC << 8  # ELU


def timeit(fn, reps=20, replays=10):
    """GPU time per launch: `reps` launches captured in a HIP graph, replayed
    (eager ctypes launches would measure the host, not the kernel)."""
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * replays) * 1e3


def floor():
    """launch floor: a tiny kernel of this library vs a tiny torch kernel"""
    L = nat.lib()
    dev = torch.device("cuda")
    x = torch.randn(1, 64, device="cuda")
    y = torch.empty_like(x)
    m = torch.empty(1, device="cuda")
    t_lib = timeit(lambda: L.td7_avgl1norm_fwd(nat.ptr(x), nat.ptr(y), nat.ptr(m), 1, 64, 1e-8, nat.stream_ptr(dev)))
    t_torch = timeit(lambda: x.add_(1.0))
    print(f"launch floor in a graph: libexo_amd tiny kernel {t_lib:.2f} us, torch tiny kernel {t_torch:.2f} us")


def main():
    floor()
    print("MFMA operands:", os.environ.get("DB_PREC", "fp32"))
    L = nat.lib()
    dev = torch.device("cuda")
    print(f"{'M':>5} {'N':>4} {'K':>4} | {'fwd':>7} {'bwd_d':>7} {'bwd_w':>7} | {'torch fwd':>9} | GF/s fwd")
    shapes = [(1024, 300, 16), (1024, 300, 128), (1024, 300, 256), (1024, 300, 512), (256, 32, 128), (32, 32, 128),
              (32, 32, 1024)] if os.environ.get("DB_SWEEP") else []
    for (m, n, k) in shapes + [(1024, 300, 80), (1024, 300, 300), (1024, 300, 307), (1024, 320, 620), (1024, 320, 920),
                      (1024, 7, 320), (4096, 300, 300), (2048, 300, 300)]:
        x = torch.randn(m, k, device="cuda")
        w = torch.randn(n, k, device="cuda")
        b = torch.randn(n, device="cuda")
        y = torch.empty(m, n, device="cuda")
        dy = torch.randn(m, n, device="cuda")
        dx = torch.empty(m, k, device="cuda")
        dw = torch.empty(n, k, device="cuda")
        db = torch.empty(n, device="cuda")
        P = nat.ptr
        f = timeit(lambda: L.td7_dense_fwd(P(x), 0, k, P(w), P(b), P(y), m * n, n, 1, m, n, k, ACT, nat.stream_ptr(dev)))
        bd = timeit(lambda: L.td7_dense_bwd_data(P(dy), m * n, n, P(y), m * n, n, P(w), P(dx), m * k, k, 1, 0,
                                                  m, n, k, ACT, nat.stream_ptr(dev)))
        bw = timeit(lambda: L.td7_dense_bwd_weight(P(dy), m * n, n, P(y), m * n, n, P(x), 0, k, P(dw), P(db), 1,
                                                    m, n, k, ACT, nat.stream_ptr(dev)))
        tf = timeit(lambda: torch.nn.functional.elu(torch.nn.functional.linear(x, w, b)))
        print(f"{m:5d} {n:4d} {k:4d} | {f:7.2f} {bd:7.2f} {bw:7.2f} | {tf:9.2f} | {2 * m * n * k / f / 1e3:8.0f}")
    # the critic's two Q heads: groups = 2, separate inputs (TD7 critic q2/q3 layers)
    for (m, n, k) in [(1024, 320, 920), (1024, 320, 320)]:
        x = torch.randn(2, m, k, device="cuda")
        w = torch.randn(2, n, k, device="cuda")
        b = torch.randn(2, n, device="cuda")
        y = torch.empty(2, m, n, device="cuda")
        dy = torch.randn(2, m, n, device="cuda")
        dx = torch.empty(2, m, k, device="cuda")
        dw = torch.empty(2, n, k, device="cuda")
        db = torch.empty(2, n, device="cuda")
        P = nat.ptr
        f = timeit(lambda: L.td7_dense_fwd(P(x), m * k, k, P(w), P(b), P(y), m * n, n, 2, m, n, k, ACT, nat.stream_ptr(dev)))
        bd = timeit(lambda: L.td7_dense_bwd_data(P(dy), m * n, n, P(y), m * n, n, P(w), P(dx), m * k, k, 2, 0,
                                                  m, n, k, ACT, nat.stream_ptr(dev)))
        bw = timeit(lambda: L.td7_dense_bwd_weight(P(dy), m * n, n, P(y), m * n, n, P(x), m * k, k, P(dw), P(db), 2,
                                                    m, n, k, ACT, nat.stream_ptr(dev)))
        tf = timeit(lambda: torch.nn.functional.elu(torch.baddbmm(b.unsqueeze(1), x, w.transpose(1, 2))))
        print(f"2x{m:4d} {n:4d} {k:4d} | {f:7.2f} {bd:7.2f} {bw:7.2f} | {tf:9.2f} | {4 * m * n * k / f / 1e3:8.0f}")


if __name__ == "__main__":
    main()
