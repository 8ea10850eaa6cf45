"""The round-4 host crash in graph replay, as a test.

Round 4's default bench segfaulted inside hipGraphLaunch (fault address
0x1d8, libamdhip64 +0xaee41: a load through a stale hip::Stream pointer while
the runtime picks the streams of a graph's parallel branches) at the first
replay of a trainer that ran after (1) an async-episode VecTrainer -- whose
graphs hold exo_reset_list_kernel -- (2) the reference schedule with burst
prefetch and (3) its tremor-statistics rounds.  r05 bisection
(tools/bp_crash_repro.py, profiles/r05seg_raw): the same tree with round 4's
reset kernels (2,112 B/lane of scratch each) crashes, with the r05 reset
kernels (16 envs per workgroup, 144 B/lane) it runs clean.  This test builds
that combination at the bench's size and checks the last trainer trains."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_trainer_after_async_trainer_and_burst_prefetch_stats_rounds(monkeypatch):
    from exo_amd import VecExoskeletonEnv
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
    for _ in range(150):
        tr0.step()
    torch.cuda.synchronize()
    assert tr0.graphs
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
    retire_graphs(tr1)  # the mitigation: its graph execs stay alive (exo_amd.rollout.retire_graphs)
    del tr1, ag1
    torch.cuda.synchronize()
    ag2 = agent()
    tr2 = VecTrainer(env, ag2, episodes="sync")  # the trainer whose first replay crashed in r04
    for _ in range(60):
        tr2.step()
    torch.cuda.synchronize()
    assert len(tr2.graphs) == 2
    for m in (ag2.learner.actor, ag2.learner.critic, ag2.learner.encoder):
        assert all(torch.isfinite(p).all() for p in m.parameters())
