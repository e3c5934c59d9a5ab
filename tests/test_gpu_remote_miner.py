"""Remote-mode mining on the MI355X: the GPU backend (per-period HIP kernel, DAG in HBM) mining
for a regtest node through getblocktemplate / pprpcsb, every share host re-verified."""
import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures

pytestmark = pytest.mark.gpu


def test_gpu_remote_miner(gpu, core, node_factory):  # noqa: F811
    from nodexa_chain_core_amd.miner.remote import RemoteMiner
    from nodexa_chain_core_amd.miner.search import GpuSearchDevice

    node, _ = node_factory()
    c = client(node)
    m = RemoteMiner(c, GpuSearchDevice(0), window=1 << 16, rank=2)
    stats = m.run(max_blocks=3, max_seconds=180)
    assert stats["accepted"] == 3 and stats["rejected"] == 0, stats
    assert c.getblockcount() == 3
