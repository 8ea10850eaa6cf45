"""RCCL world-1 in-graph layout vs the one-GPU graph (tests/test_dp_gpu.py::
test_rccl_inline_layout_is_bit_identical_to_the_one_gpu_graph), in a process of
its own.  usage: python tests/rccl_inline_worker.py PORT -> prints OK."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))

import torch  # noqa: E402


class _Env:
    """monkeypatch.setenv's stand-in"""

    @staticmethod
    def setenv(k, v):
        os.environ[k] = v


def _port():
    return int(sys.argv[1])


monkeypatch = _Env()


def main():
    import torch.distributed as dist
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters

    def run(group, capture="1", planned=False):
        monkeypatch.setenv("EXO_FORCE_DIST", "1" if group is not None else "0")
        monkeypatch.setenv("EXO_DP_CAPTURE", capture)
        torch.manual_seed(11)
        env = VecExoskeletonEnv(512, seed=21)
        ag = Agent(80, 7, 1, env_num=8, precision="bf16", n_envs=512, process_group=group, graph_safe=True,
                   buffer_size=8192, hp=Hyperparameters(target_update_rate=5))
        tr = VecTrainer(env, ag)
        if planned:  # the overlapped pairs (r05), collectives captured inside them
            tr.plan(14)
        for _ in range(14):
            tr.step()
        torch.cuda.synchronize()
        L = ag.learner
        st = [p.detach().clone() for m in (L.actor, L.critic, L.encoder, L.fixed_encoder) for p in m.parameters()]
        st += [getattr(L, o).m.clone() for o in ("actor_optimizer", "critic_optimizer", "encoder_optimizer")]
        st += [ag.replay_buffer._tree.clone(), ag.replay_buffer._maxp.clone(), L.max.clone(), L.min.clone()]
        return tr, st

    tr0, ref = run(None)
    assert not tr0.dp
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        for capture, inline, planned in (("1", True, False), ("1", True, True), ("0", False, False)):
            tr, st = run(dist.group.WORLD, capture, planned)
            assert tr.dp and tr.dp_inline is inline
            if inline:  # the extended captured-collective self-test (GradSync._capture_selftest) ran and passed
                assert tr.agent.sync._capture_ok is True
                assert all(len(parts) == 1 for k, parts in tr.graphs.items() if k[0] != "pair")
                assert any(k[-1] == "overlap" for k in tr.graphs) == planned
                assert tr._refresh_graph is not None
            for i, (x, y) in enumerate(zip(ref, st)):
                torch.testing.assert_close(y, x, rtol=0, atol=0, msg=f"tensor {i} (capture={capture}, pairs={planned})")
    finally:
        dist.destroy_process_group()
    print("OK")


if __name__ == "__main__":
    main()
