"""Graph lifetime and the ROCm 7.0 graph-launch fault.

The fault: a graph exec owns one runtime stream per parallel branch; the
runtime assigns them at every launch, skipping a stream on the launch
stream's hardware queue, with no bound on the stream index.  Destroyed execs
release their streams unevenly; once the launch queue is the least loaded by
two, a new exec gets two streams there and its launch reads past its stream
vector (libamdhip64 +0xaee41 from +0xaf924).  tools/graph_stream_pool_repro.hip
reproduces it without torch (profiles/r06_graph_fault: "destroy" faults at
trial 38, "keep" and "ballast" run clean).  exo_amd.graphs.release_graphs
destroys graphs and then creates ballast streams (at least as many as the
execs held: new streams go to the least-loaded queue, so the loads are even
again); these tests run the launch patterns that faulted through it."""
import random

import pytest
import torch

pytestmark = pytest.mark.gpu


def _forked_graph(side, branches, ctr):
    """A root on the capture stream side[0], branches - 1 forked side streams
    side[1:] each adding into its own counter slot, joined back (the repro's
    shapes).  The five streams are taken once: torch's stream pool hands the
    same 32 streams out in turn, so a new one per call would alias a side
    stream and merge two branches."""
    from exo_amd.graphs import capture, new_graph
    s, side = side[0], side[1:]
    s.wait_stream(torch.cuda.current_stream())
    g = new_graph()
    with torch.cuda.stream(s):
        with capture(g, stream=s):
            ctr[0].add_(1)
            for b in range(1, branches):
                side[b - 1].wait_stream(s)
                with torch.cuda.stream(side[b - 1]):
                    ctr[b].add_(1)
            ctr[0].add_(1)  # the capture stream's own branch
            for b in range(1, branches):
                s.wait_stream(side[b - 1])
            ctr[7].add_(1)
    torch.cuda.current_stream().wait_stream(s)
    return g


def test_release_graphs_keeps_later_launches_safe():
    """The torch-free repro's "destroy" pattern (1-3 new execs per trial, a
    random half of the live ones destroyed, every live one launched), in this
    process through release_graphs: no fault over 120 trials, every branch ran
    as often as launched, and each forked graph's branch bound counts its
    branches."""
    from exo_amd.graphs import branch_bound, release_graphs
    rng = random.Random(1)
    side = [torch.cuda.Stream() for _ in range(5)]
    ctr = torch.zeros(8, dtype=torch.int64, device="cuda")
    want = [0] * 8
    live = []
    for t in range(120):
        for _ in range(1 + rng.randrange(3)):
            b = 2 + rng.randrange(4)
            g = _forked_graph(side, b, ctr)
            assert branch_bound(g) >= b
            live.append((g, b))
        gone = [x for x in live if rng.random() < 0.5] if len(live) > 1 else []
        if len(gone) == len(live):
            gone = gone[1:]
        if gone:
            assert release_graphs([g for g, _ in gone]) == len(gone)
            live = [x for x in live if all(x is not y for y in gone)]
        for g, b in live:
            g.replay()
            want[0] += 2
            for k in range(1, b):
                want[k] += 1
            want[7] += 1
        torch.cuda.synchronize()
    assert ctr.tolist() == want
    release_graphs([g for g, _ in live])


def test_trainer_after_async_trainer_and_burst_prefetch_stats_rounds(monkeypatch):
    """Round 4's crash combination at the bench's size -- an async-episode
    VecTrainer, the reference schedule with burst prefetch and its
    tremor-statistics rounds -- each trainer released (execs and memory pools
    destroyed, ballast streams) before the next, then a new trainer's first
    replays (where r04 faulted): it trains, and the released trainers' graph
    memory is returned."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.graphs import kept_graphs
    from exo_amd.rollout import RefScheduleTrainer, VecTrainer, retire_graphs
    from exo_amd.td7 import Agent, Hyperparameters
    monkeypatch.setenv("EXO_BURST_PREFETCH", "1")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    env = VecExoskeletonEnv(4096, seed=1000, device=dev)

    def agent():
        return Agent(80, 7, 1, env_num=8, hp=Hyperparameters(), device=dev, precision="bf16", n_envs=4096,
                     graph_safe=True)
    ag0 = agent()
    tr0 = VecTrainer(env, ag0, episodes="async")  # (1): resets inside its graphs
    tr0.plan(150)
    for _ in range(150):
        tr0.step()
    torch.cuda.synchronize()
    assert tr0.graphs
    k0 = kept_graphs()
    assert retire_graphs(tr0) > 0
    assert kept_graphs() < k0
    del tr0, ag0
    ag1 = agent()
    tr1 = RefScheduleTrainer(env, ag1, warmup=25_000)  # (2) burst prefetch
    assert tr1.burst_prefetch
    for _ in range(6):
        tr1.run_round()
    tr1.stats = True  # (3) the tremor-statistics rounds
    for _ in range(3):
        tr1.run_round()
    torch.cuda.synchronize()
    assert any(k[0] == "train" and len(k) == 5 for k in tr1.graphs)  # prefetching burst graphs were replayed
    assert len(tr1.round_stats) == 3
    torch.cuda.empty_cache()
    held = torch.cuda.memory_reserved(dev)
    assert retire_graphs(tr1) > 0  # execs and pools destroyed, ballast streams created
    del tr1, ag1
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    assert torch.cuda.memory_reserved(dev) < held  # the graph pools were returned
    ag2 = agent()
    tr2 = VecTrainer(env, ag2, episodes="sync")  # the trainer whose first replay crashed in r04
    for _ in range(60):
        tr2.step()
    torch.cuda.synchronize()
    assert len(tr2.graphs) == 2
    for m in (ag2.learner.actor, ag2.learner.critic, ag2.learner.encoder):
        assert all(torch.isfinite(p).all() for p in m.parameters())
