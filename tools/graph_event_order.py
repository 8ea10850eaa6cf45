"""Does an event recorded on a stream after a HIP graph replay order a second
stream's work after the graph?  (gloo's CUDA all-reduce and RCCL both rely on
it.)  Prints the number of stale reads out of `trials`."""
import torch


def simple_graph_check(trials=20, n=1 << 24, reps=40):
    x = torch.zeros(n, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    x.zero_()
    other = torch.cuda.Stream(priority=-1)  # gloo and RCCL use high-priority pool streams
    host = torch.empty(n, pin_memory=True)
    bad_event = bad_wait = 0
    for t in range(1, trials + 1):
        g.replay()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        other.wait_event(ev)
        with torch.cuda.stream(other):
            host.copy_(x, non_blocking=True)
        other.synchronize()
        bad_event += int(float(host[-1]) != reps * t)
        # same via wait_stream
        torch.cuda.synchronize()
    x.zero_()
    for t in range(1, trials + 1):
        g.replay()
        other.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(other):
            host.copy_(x, non_blocking=True)
        other.synchronize()
        bad_wait += int(float(host[-1]) != reps * t)
        torch.cuda.synchronize()
    print(f"stale reads after graph replay: event {bad_event}/{trials}, wait_stream {bad_wait}/{trials}")
    return bad_event + bad_wait


def trainer_graph_check(iters=12):
    """Same question on the real training graphs: after replaying the
    'pre' graph of the data-parallel layout, read its flat gradient bucket
    from another stream ordered only by an event."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent
    env = VecExoskeletonEnv(256, seed=5)
    agent = Agent(80, 7, 1, env_num=8, n_envs=256, graph_safe=True)
    tr = VecTrainer(env, agent)
    tr.dp = True
    for _ in range(6):
        tr.step()
    torch.cuda.synchronize()
    other = torch.cuda.Stream(priority=-1)  # gloo and RCCL use high-priority pool streams
    bad = 0
    for it in range(iters):
        par = it % 2 == 0
        g1, g2, g3, flat_c, flat_a = next(v for k, v in tr.graphs.items() if k[0] == par)
        host = torch.empty(flat_c.numel(), pin_memory=True)
        g1.replay()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        other.wait_event(ev)
        with torch.cuda.stream(other):
            host.copy_(flat_c, non_blocking=True)
        other.synchronize()
        torch.cuda.synchronize()
        ref = flat_c.cpu()
        bad += int(not torch.equal(host, ref))
        g2.replay()
        if g3 is not None:  # captured only at the actor-update parity
            g3.replay()
        torch.cuda.synchronize()
    print(f"trainer 'pre' graph: stale/racy bucket reads {bad}/{iters}")
    return bad


if __name__ == "__main__":
    simple_graph_check()
    trainer_graph_check()
