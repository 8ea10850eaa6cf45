"""Fork/join discipline of the captured iteration: every
stream forked from the capture stream must join back before capture end
(exo_amd/rollout.py unjoined_streams / ForkJoinAudit, applied to every capture
VecTrainer makes)."""
import pytest


class S:
    def __init__(self, h):
        self.cuda_stream = h


def _unjoined(events, origin):
    from exo_amd.rollout import unjoined_streams
    return {s.cuda_stream for s in unjoined_streams(events, origin)}


def test_fork_join_patterns():
    o, a, b, c = S(1), S(2), S(3), S(4)
    # fork a, work on a, join a: clean
    assert _unjoined([("wait", a, o), ("use", a), ("wait", o, a)], o) == set()
    # fork without join
    assert _unjoined([("wait", a, o), ("use", a)], o) == {2}
    # joined, then more work enqueued on the branch: unjoined
    assert _unjoined([("wait", a, o), ("use", a), ("wait", o, a), ("use", a)], o) == {2}
    # a re-fork after the join (reused side stream) that is joined again: clean
    ev = [("wait", a, o), ("use", a), ("wait", o, a), ("wait", a, o), ("use", a), ("wait", o, a)]
    assert _unjoined(ev, o) == set()
    # transitive: b forks from a, joins into a, a joins into origin afterwards
    ev = [("wait", a, o), ("wait", b, a), ("use", b), ("use", a), ("wait", a, b), ("wait", o, a)]
    assert _unjoined(ev, o) == set()
    # transitive join that happens before the branch's last use does not count
    ev = [("wait", a, o), ("wait", b, a), ("wait", a, b), ("wait", o, a), ("use", b)]
    assert _unjoined(ev, o) == {3}
    # a stream never forked from the capture is not a branch of it
    assert _unjoined([("wait", c, S(9)), ("use", c)], o) == set()


@pytest.mark.gpu
def test_forgotten_join_is_reported_and_capture_survives():
    import torch
    from exo_amd.rollout import CaptureForkError, ForkJoinAudit
    s, br = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.zeros(16, device="cuda")
    s.wait_stream(torch.cuda.current_stream())
    from exo_amd.graphs import new_graph
    g = new_graph()
    with torch.cuda.stream(s):
        with pytest.raises(CaptureForkError):
            with torch.cuda.graph(g, stream=s), ForkJoinAudit(s):
                x.add_(1)
                br.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(br):
                    x.mul_(2)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 2.0  # (0 + 1) * 2: the audit joined the branch, capture ended cleanly


@pytest.mark.gpu
@pytest.mark.parametrize("prio_branch", [True, False])
def test_trainer_captures_are_fork_join_clean(prio_branch, monkeypatch):
    import torch
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    hp = Hyperparameters(zs_dim=64, enc_hdim=64, critic_hdim=64, actor_hdim=64, batch_size=32)
    env = VecExoskeletonEnv(64, seed=3)
    agent = Agent(80, 7, 1, hp=hp, env_num=8, device="cuda:0", buffer_size=4096, precision="bf16")
    monkeypatch.setattr(VecTrainer, "prio_branch", prio_branch)
    tr = VecTrainer(env, agent, warmup_eager=2)
    for _ in range(8):  # eager warm-up, then both parities captured under the audit and replayed
        tr.step()
    torch.cuda.synchronize()
    assert len(tr.graphs) >= 2


def test_audit_is_reentrant_and_thread_scoped(monkeypatch):
    """nested audits unpatch only when the outermost exits, and an
    audit records only its own thread's waits (CPU: the torch methods are
    replaced by stubs first, so no stream is needed)."""
    import threading

    import torch
    from exo_amd.rollout import ForkJoinAudit
    calls = []
    monkeypatch.setattr(torch.cuda.Stream, "wait_stream", lambda st, other: calls.append((st, other)))
    stub_wait = torch.cuda.Stream.wait_stream
    o, a, b = S(1), S(2), S(3)
    outer, inner = ForkJoinAudit(o), ForkJoinAudit(o)
    with outer:
        torch.cuda.Stream.wait_stream(a, o)
        with inner:
            torch.cuda.Stream.wait_stream(o, a)
            t = threading.Thread(target=lambda: torch.cuda.Stream.wait_stream(b, o))  # not ours
            t.start()
            t.join()
        assert torch.cuda.Stream.wait_stream is not stub_wait  # still patched for the outer audit
    assert torch.cuda.Stream.wait_stream is stub_wait  # restored once the outermost exits
    assert [e[1:] for e in outer.events] == [(a, o), (o, a)]
    assert [e[1:] for e in inner.events] == [(o, a)]
    assert len(calls) == 3  # every call reached the original method
