"""LAP launch timings at the bench's shape (8 strata x 250,000 slots, 176,128
transitions per stratum -- one 4,096-env episode round -- batch 8 x 128): the
training loop's priority update + next sample (one launch), and the update /
sample-gather launches alone.  Each launch captured 20x in a HIP graph, timed
with HIP events over 10 replays.  usage: python tools/lap_bench.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import torch  # noqa: E402


def timed(fn, reps=20, replays=10):
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


def main():
    from exo_amd.replay import LAP
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    rb = LAP(80, 7, dev, 8, 250_000, 128)
    n = 4096
    strata = (torch.arange(n, device=dev) % 8).to(torch.int32)
    obs = torch.randn(n, 80, device=dev)
    act = torch.rand(n, 7, device=dev) * 2 - 1
    rew = torch.rand(n, device=dev)
    done = torch.zeros(n, dtype=torch.bool, device=dev)
    for _ in range(344):
        rb.add_batch(obs, act, obs, rew, done, strata)
    rb.sample(0)
    torch.cuda.synchronize()
    ind = rb.ind.clone()
    prio = torch.rand(8 * 128, device=dev) * 3

    def upd_sample():
        rb.update_priority_and_sample(prio, ind, slot=1)

    def upd():
        rb.update_priority(prio, ind)

    def smp():
        rb.sample(1)
    # the reference schedule's per-step insert (shared pointer) with the mask advance, on a second buffer
    rb2 = LAP(80, 7, dev, 8, 250_000, 128)
    table = torch.ones((345, n), dtype=torch.bool, device=dev)
    k = torch.zeros((1,), dtype=torch.int64, device=dev)
    active = torch.ones(n, dtype=torch.bool, device=dev)
    count = torch.zeros((1,), dtype=torch.int32, device=dev)
    score = torch.zeros(n, dtype=torch.float64, device=dev)

    def ref_insert():
        rb2.add_batch_ref(obs, act, obs, rew, done, strata, active, advance=(table, k, count, score))
    for name, f in (("update + sample (one launch)", upd_sample), ("update alone", upd), ("sample + gather", smp),
                    ("ref insert + mask advance", ref_insert)):
        print(f"{name:32s} {timed(f):8.2f} us", flush=True)


if __name__ == "__main__":
    main()
