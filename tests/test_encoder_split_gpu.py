"""td7f_encoder with zs(next_state) on its own workgroup row (r04, VERDICT r3
item 2): the producer row publishes next_zs through global memory and a
per-tile flag, the consumer row runs zs(s), zsa and the backward and reads it
at the mse gradient.  The split pass must leave exactly the outputs of the
one-row pass -- the saved activations, every transposed weight-gradient
operand and its column partials -- eagerly, again on a second launch (the
flags are cleared by the consumer), and from a replayed HIP graph; and the
flags must be left zero."""
import pytest
import torch

from exo_amd.td7 import Hyperparameters, TD7Learner

pytestmark = pytest.mark.gpu


def _outputs(tr):
    out = [t.clone() for t in tr.y_enc]
    for xb in tr.xt_enc:
        out += [xb.x.clone(), xb.dp.clone(), xb.part.clone()]
    return out


@pytest.mark.parametrize("precision,width,B", [("bf16", None, 1024), ("fp16", 256, 1000), ("bf16", None, 40)])
def test_split_encoder_pass_is_bit_identical(precision, width, B):
    torch.manual_seed(3)
    hp = Hyperparameters() if width is None else Hyperparameters(zs_dim=width, enc_hdim=width, critic_hdim=width,
                                                                 actor_hdim=width)
    L = TD7Learner(80, 7, hp, device="cuda", precision=precision)
    assert L.fused is not None
    tr = L.fused.train(B)
    g = torch.Generator(device="cuda").manual_seed(5)
    s = torch.randn(B, 80, device="cuda", generator=g)
    a = torch.rand(B, 7, device="cuda", generator=g) * 2 - 1
    ns = torch.randn(B, 80, device="cuda", generator=g)
    tr.enc_split = False
    tr.encoder(s, a, ns)
    want = _outputs(tr)
    tr.enc_split = True
    for _ in range(2):
        for t in _outputs(tr):
            t.zero_()
        tr.encoder(s, a, ns)
        torch.cuda.synchronize()
        for i, (x, y) in enumerate(zip(want, _outputs(tr))):
            torch.testing.assert_close(y, x, rtol=0, atol=0, msg=f"output {i}")
        assert int(tr.enc_flag.abs().sum()) == 0
    # graph-captured: three launches per replay, three replays
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    from exo_amd.graphs import new_graph
    gr = new_graph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(gr, stream=st):
            for _ in range(3):
                tr.encoder(s, a, ns)
    torch.cuda.current_stream().wait_stream(st)
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip(want, _outputs(tr))):
        torch.testing.assert_close(y, x, rtol=0, atol=0, msg=f"replayed output {i}")
    assert int(tr.enc_flag.abs().sum()) == 0
