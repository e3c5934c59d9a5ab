"""Persistent block index (chain/blockindex.py, the CBlockTreeDB role): restart without
re-reading blk files, torn-tail truncation, recovery of blocks written after the last
index record, and -reindex (mirrors the reference's feature_reindex.py and the
crash-recovery half of feature_dbcrash.py)."""
import os

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures


def _index(node):
    return os.path.join(node.datadir, "blocks", "index.log")


def test_restart_from_index_and_recovery(core, node_factory):  # noqa: F811
    from nodexa_chain_core_amd.chain.blockindex import BlockIndexLog

    node, addr = node_factory(["-dbformat=journal"])
    c = client(node)
    hashes = c.generatetoaddress(5, addr)
    path = _index(node)
    node.stop()
    recs = BlockIndexLog(path).load()
    assert len(recs) == 6  # genesis + 5

    # 1. clean restart: tip and block bodies come back from the index records
    node, _ = node_factory()
    c = client(node)
    assert c.getbestblockhash() == hashes[-1] and c.getblock(hashes[2])["height"] == 3
    node.stop()

    # 2. torn final record: cut off on load, the block is recovered from the blk-file tail
    size = os.path.getsize(path)
    with open(path, "r+b") as f:
        f.truncate(size - 7)
    node, _ = node_factory()
    c = client(node)
    assert c.getbestblockhash() == hashes[-1]
    node.stop()
    assert len(BlockIndexLog(path).load()) == 6

    # 3. garbage appended (crash mid-write): ignored and truncated
    with open(path, "ab") as f:
        f.write(b"\x30\x00\x00\x00garbage")
    node, _ = node_factory()
    c = client(node)
    assert c.getblockcount() == 5
    c.generatetoaddress(1, addr)
    node.stop()
    assert len(BlockIndexLog(path).load()) == 7

    # 4. -reindex: rebuilt from the blk files, index rewritten
    os.remove(path)
    node, _ = node_factory(("-reindex",))
    c = client(node)
    assert c.getblockcount() == 6 and c.getblockhash(5) == hashes[-1]
    node.stop()
    assert len(BlockIndexLog(path).load()) == 7
