"""Reproduce the burst-prefetch crash outside bench.py: a reference-schedule
trainer with EXO_BURST_PREFETCH=1 runs 6 rounds at 4,096 envs, then a fresh
VecTrainer (sync episodes) on the same env (or, with argv[1] == "newenv", a
new env) captures and replays its graphs.  argv[2]: rounds (default 6)."""
import os
import sys

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402

# diagnostics (r05): a native SIGSEGV backtrace with per-library offsets
import ctypes  # noqa: E402
import faulthandler  # noqa: E402
import traceback  # noqa: E402

faulthandler.enable()
_tr = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_segv_trace.so")
if os.path.exists(_tr):
    ctypes.CDLL(_tr).segv_trace_install()


def _bisect_switches():
    """r05 bisection of the two r05 changes that made the crash go away:
    "r04reset" loads a library built with round 4's reset kernels (one
    wavefront per env, 2,112 B/lane of scratch), made from the r04 source:
      git show b3aefae:<pkg>/csrc/exo_env.hip > tools/_bisect/exo_env_r04.hip
      (cd <pkg>/csrc && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC
       -I../../include -I. -c ../../tools/_bisect/exo_env_r04.hip -o ../../tools/_bisect/exo_env_r04.o &&
       hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_bisect/libexo_amd_r04reset.so
       ../../tools/_bisect/exo_env_r04.o <every other ../exo_amd/_lib/*.o>)
    "r04select" passes the select workgroup cap by setting EXO_SELECT_WG_CAP
    in os.environ around every td7f_select call, as round 4 did."""
    import exo_amd._native as nat
    from exo_amd import fused
    if "r04reset" in sys.argv:
        nat.LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_bisect", "libexo_amd_r04reset.so")
        print("library", nat.LIB_PATH, flush=True)
    if "r04select" in sys.argv:
        orig = fused.FusedNets.select

        def select(self, obs, scale=1.0, dec_count=None, world=1, wg_cap=None):
            prev = os.environ.get("EXO_SELECT_WG_CAP")
            if wg_cap is not None:
                os.environ["EXO_SELECT_WG_CAP"] = str(int(wg_cap))
            try:
                return orig(self, obs, scale, dec_count, world, None)
            finally:
                if wg_cap is not None:
                    if prev is None:
                        del os.environ["EXO_SELECT_WG_CAP"]
                    else:
                        os.environ["EXO_SELECT_WG_CAP"] = prev
        fused.FusedNets.select = select
        print("select cap through os.environ", flush=True)


def main():
    _bisect_switches()
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer, VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    mode = sys.argv[1] if len(sys.argv) > 1 else "same"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda", 0)
    env = VecExoskeletonEnv(4096, seed=1000, device=dev)
    keep = None
    if "main" in sys.argv:  # the bench's own trainer first, alive through the rest
        ag0 = Agent(80, 7, 1, env_num=8, hp=Hyperparameters(), device=dev, precision="bf16", n_envs=4096,
                    graph_safe=True)
        tr0 = VecTrainer(env, ag0, episodes="async")
        for _ in range(150):
            tr0.step()
        torch.cuda.synchronize()
        keep = (tr0, ag0)
        print("main trainer graphs", len(tr0.graphs), flush=True)
        if "release_main" in sys.argv:  # the live-graph-count hypothesis
            tr0.graphs.clear()
            torch.cuda.synchronize()
            print("main trainer graphs released", flush=True)
    ag = Agent(80, 7, 1, env_num=8, hp=Hyperparameters(), device=dev, precision="bf16", n_envs=4096, graph_safe=True)
    tr = RefScheduleTrainer(env, ag, warmup=25_000)
    print("burst_prefetch", tr.burst_prefetch, flush=True)
    for r in range(rounds):
        tr.run_round()
        print("round", r, "graphs", len(tr.graphs), sorted(map(str, tr.graphs))[:3], flush=True)
    if "stats" in sys.argv:  # the bench's tremor-statistics rounds
        tr.stats = True
        for r in range(3):
            tr.run_round()
            print("stats round", r, "graphs", len(tr.graphs), flush=True)
    torch.cuda.synchronize()
    keys = sorted(map(str, tr.graphs))
    print("ref trainer graph keys:", keys, flush=True)
    if "retire" in sys.argv:  # r05 mitigation: keep the finished trainer's graph execs alive
        from exo_amd.rollout import retire_graphs
        retire_graphs(tr)
        print("graphs retired", flush=True)
    del tr, ag
    import gc
    gc.collect()
    torch.cuda.synchronize()
    if mode == "newenv":
        env = VecExoskeletonEnv(4096, seed=1001, device=dev)
    ag2 = Agent(80, 7, 1, env_num=8, hp=Hyperparameters(), device=dev, precision="bf16", n_envs=4096,
                graph_safe=True)
    tr2 = VecTrainer(env, ag2, episodes="sync")
    for i in range(60):
        tr2.step()
        if i < 8:
            torch.cuda.synchronize()
            print("vec step", i, "graphs", len(tr2.graphs), flush=True)
    torch.cuda.synchronize()
    print("second trainer ok", flush=True)


if __name__ == "__main__":
    main()
