"""Equihash solve sequence replayed from a hipGraph (ops/equihash.py, capture_equihash_solve; the
global-slot engine): same solutions as direct launches, across several replays with new inputs in
between."""
import os

import pytest

pytestmark = pytest.mark.gpu


def test_graph_replays_match_direct_launches():
    import torch

    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    os.environ["NODEXA_EQ_GRAPH"] = "1"
    try:
        g = EquihashSolver(num_inst=4, device=0, engine="global")
    finally:
        del os.environ["NODEXA_EQ_GRAPH"]
    d = EquihashSolver(num_inst=4, device=0, engine="global")
    assert g.use_graph and not d.use_graph
    key = lambda sols: [sorted(map(tuple, s)) for s in sols]  # noqa: E731
    for rep in range(4):
        inputs = [bytes([rep * 4 + i]) * 108 + b"\x00" * 4 for i in range(4)]
        a = g.solve(inputs)  # verified against the CPU verifier inside collect()
        torch.cuda.synchronize()
        assert g._graph is not None and g._graph.num_nodes == 11
        assert key(a) == key(d.solve(inputs))
