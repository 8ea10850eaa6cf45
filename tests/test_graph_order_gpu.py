"""HIP graph properties the replayed training iteration relies on:
  * multi-block torch reductions replay correctly (needs
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=0, set by exo_amd / conftest);
  * an event recorded after a graph replay orders a collective's
    (high-priority) stream after the whole graph -- on a toy graph and on the
    real 'pre' training graph of the data-parallel layout."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_event_after_graph_replay_orders_other_stream():
    import graph_event_order as G
    assert G.simple_graph_check() == 0


def test_training_graph_bucket_complete_before_collective_stream():
    import graph_event_order as G
    assert G.trainer_graph_check() == 0


def test_graph_reductions_replay_correctly():
    import torch
    from exo_amd.rollout import graph_reductions_ok
    assert graph_reductions_ok(torch.device("cuda", 0), replays=10)
    import graph_reduce_check as R
    assert R.main(reps=10) == 0
