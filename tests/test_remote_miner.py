"""Remote-mode miner (client side): the engine mining for a node through
getblocktemplate (pprpcheader / pprpcepoch / target) and pprpcsb, as an external GPU miner does
against clore_blockchaind (src/rpc/mining.cpp:722-739, 841-932). The CPU backend runs here; the
GPU backend runs the same loop in tests/test_gpu_remote_miner.py."""
from nodexa_chain_core_amd.miner.remote import RemoteMiner
from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures


def test_remote_miner_mines_through_pprpcsb(core, node_factory):  # noqa: F811
    node, addr = node_factory()
    c = client(node)
    m = RemoteMiner(c, None, window=4096, rank=1)
    stats = m.run(max_blocks=3, max_seconds=120)
    assert stats["accepted"] == 3 and stats["rejected"] == 0
    assert c.getblockcount() == 3
    blk = c.getblock(c.getbestblockhash())
    assert int(blk["nonce64"] if isinstance(blk["nonce64"], int) else int(blk["nonce64"], 16)) >> 56 == 1  # rank 1
    # the tip moves under the miner: the next step re-reads the template instead of mining stale work
    old = m.template()["pprpcheader"]
    c.generatetoaddress(1, addr)
    assert m.template()["pprpcheader"] != old
    m.step()
    assert c.getblockcount() >= 4
