"""Do column reductions (torch sum over dim 0, the bias-gradient shape of the
TD7 nets) replay correctly from HIP graphs?  Compares each replay with an
eager recomputation; prints mismatching replays.  With the ROCm 7.2 default
(graph packet capture on) 29 of 30 replays are wrong; with
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 none are (profiles/r01_graph_reduce_check.txt)."""
import torch


def main(reps=30, n_red=24, rows=1024, cols=300):
    torch.manual_seed(0)
    xs = [torch.randn(rows, cols, device="cuda") for _ in range(n_red)]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for x in xs:  # warm
            x.sum(0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            outs = [x.sum(0) for x in xs]
            big = [torch.empty(4096, device="cuda").fill_(float("nan")) for _ in range(4)]  # garbage writers
    torch.cuda.current_stream().wait_stream(s)
    ref = [x.sum(0) for x in xs]
    bad = 0
    for r in range(reps):
        for x in xs:
            x.mul_(1.0001)
        ref = [x.sum(0) for x in xs]
        g.replay()
        if r % 2:
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        for o, e in zip(outs, ref):
            if not torch.allclose(o, e, rtol=1e-5, atol=1e-5):
                bad += 1
                nanmask = ~torch.isfinite(o)
                print(f"replay {r}: mismatch, non-finite {int(nanmask.sum())}, max diff "
                      f"{float((o - e).abs().nan_to_num(1e30).max()):.3g}", flush=True)
                break
    print(f"graph column-reduction mismatches: {bad}/{reps}")
    return bad


if __name__ == "__main__":
    import os
    main(rows=int(os.environ.get("GRC_ROWS", 1024)))
