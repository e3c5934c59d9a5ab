"""Block-file pruning (-prune, pruneblockchain; src/validation.cpp:12208-12343,
src/rpc/blockchain.cpp:1133-1180, feature_pruning.py in the reference's functional suite). The
tests shrink the blk file size and the prune-after height so a few hundred regtest blocks span
many files; MIN_BLOCKS_TO_KEEP (288) is the reference's."""
import os

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures


def _small_files(node, after=50):
    node.state.store.set_max_file_size(4000)
    node.state.prune_after_height = after


def _blk_files(node):
    d = os.path.dirname(node.state.store.path(0))
    return sorted(f for f in os.listdir(d) if f.startswith("blk"))


def test_manual_prune_and_restart(core, node_factory):  # noqa: F811
    node, addr = node_factory(("-prune=1",))
    _small_files(node)
    c = client(node)
    c.generatetoaddress(400, addr)
    info = c.getblockchaininfo()
    assert info["pruned"] is True and info["automatic_pruning"] is False and info["pruneheight"] == 0
    assert "prune_target_size" not in info
    assert int(c.getnetworkinfo()["localservices"], 16) & 1 == 0  # no NODE_NETWORK
    n_files = len(_blk_files(node))
    assert n_files > 10
    with pytest.raises(RuntimeError, match="shorter than the attempted prune height"):
        c.pruneblockchain(1000)
    with pytest.raises(RuntimeError, match="Negative block height"):
        c.pruneblockchain(-1)
    assert c.pruneblockchain(100) == 100
    ph = c.getblockchaininfo()["pruneheight"]
    assert 0 < ph <= 101
    assert len(_blk_files(node)) < n_files and "blk00000.dat" not in _blk_files(node)
    with pytest.raises(RuntimeError, match="pruned data"):
        c.getblock(c.getblockhash(5))
    assert c.getblock(c.getblockhash(ph))["height"] == ph
    assert c.getblockheader(c.getblockhash(5))["height"] == 5  # headers stay
    assert c.pruneblockchain(390) == 400 - 288  # clamped to MIN_BLOCKS_TO_KEEP below the tip
    ph2 = c.getblockchaininfo()["pruneheight"]
    assert ph < ph2 <= 113
    h = c.getbestblockhash()
    node.stop()

    node, addr = node_factory(("-prune=1",))
    _small_files(node)
    c = client(node)
    assert c.getbestblockhash() == h and c.getblockchaininfo()["pruneheight"] == ph2
    c.generatetoaddress(5, addr)  # new blocks go after the last file, not into a pruned gap
    assert c.getblock(c.getbestblockhash())["height"] == 405
    assert c.gettxoutsetinfo()["height"] == 405
    node.stop()
    with pytest.raises(SystemExit, match="unpruned mode"):
        node_factory()


def test_automatic_prune_keeps_recent_blocks(core, node_factory):  # noqa: F811
    node, addr = node_factory(("-prune=550",))
    info = client(node).getblockchaininfo()
    assert info["automatic_pruning"] is True and info["prune_target_size"] == 550 << 20
    _small_files(node)
    node.state.prune_target = 20_000  # far below the files: every file old enough goes
    c = client(node)
    c.generatetoaddress(420, addr)
    tip = c.getblockcount()
    ph = c.getblockchaininfo()["pruneheight"]
    assert 0 < ph <= tip - 288 + 1
    for hgt in (tip, tip - 287):
        assert c.getblock(c.getblockhash(hgt))["height"] == hgt


@pytest.mark.parametrize("flags, msg", [(("-prune=10",), "below the minimum"),
                                        (("-prune=1", "-txindex"), "incompatible with -txindex"),
                                        (("-prune=-1",), "negative")])
def test_prune_flag_errors(core, node_factory, flags, msg):  # noqa: F811
    with pytest.raises(SystemExit, match=msg):
        node_factory(flags)
