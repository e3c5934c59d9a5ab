"""Equihash(200,9) mined through the node (the extension of SURVEY Appendix D; the reference has no
Equihash, so the flows mirrored are its KawPow ones: generateBlocks src/rpc/mining.cpp:117-173,
getblocktemplate :722-739, submitblock :934-1007, pprpcsb :841-932).

CPU devices here (the golden solver, ~2.3 s per nonce): the regtest node with `-equihash=<time>`
mines through generatetoaddress / setgenerate, an external solver takes the template's input and
answers with equihashsubmit or a full submitblock, a gloo world of 2 ranks mines Equihash blocks
with the loop's collectives, and the remote miner mines them through the RPC pair. The GPU twin
is tests/test_gpu_equihash_mining.py."""
import json
import time

import pytest

from test_miner_service import _run_world
from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures


def _eq_node(node_factory):  # noqa: F811
    return node_factory(("-equihash=%d" % (int(time.time()) - 100),))


def test_node_generates_equihash_blocks(core, node_factory):  # noqa: F811
    node, addr = _eq_node(node_factory)
    c = client(node)
    hashes = c.generatetoaddress(5, addr)
    assert len(hashes) == 5 and c.getblockcount() == 5
    act = node.params.kawpow_activation_time
    p = core.EquihashParams(200, 9)
    for h in hashes:
        b = core.Block.deserialize(bytes.fromhex(c.getblock(h, 0)), act)
        hdr = b.header
        assert hdr.is_equihash() and hdr.version & core.EQUIHASH_VERSION_BIT
        assert core.equihash_verify(p, hdr.equihash_input(), core.equihash_unpack(p, hdr.solution))[0]
        assert core.u256_hex(hdr.equihash_hash(act)) == h  # the block hash is SHA256d of the extended header
    info = c.getmininginfo()
    assert info["gpus"][0]["algo"] == "equihash" and info["gpus"][0]["blocks"] == 5
    assert info["gpus"][0]["solutionspersec"] >= 0
    # setgenerate keeps mining Equihash blocks in the background
    c.setgenerate(True)
    deadline = time.time() + 120
    while c.getblockcount() < 6 and time.time() < deadline:
        time.sleep(0.2)
    c.setgenerate(False)
    assert c.getblockcount() >= 6


def _solve_for_target(core, prefix: bytes, target: int, first_nonce: int = 1):
    """An external solver: nonce256 values until a solution's SHA256d(header) meets the target."""
    from nodexa_chain_core_amd.miner.search import equihash_block_hash, equihash_nonce256

    p = core.EquihashParams(200, 9)
    for n in range(first_nonce, first_nonce + 64):
        sols, _ = core.equihash_solve_cpu(p, prefix + equihash_nonce256(n), 16, 0)
        for s in sols:
            packed = core.equihash_pack(p, s)
            if int.from_bytes(equihash_block_hash(prefix, n, packed), "little") <= target:
                return equihash_nonce256(n), packed
    raise AssertionError("no solution met the target in 64 nonces")


def test_getblocktemplate_equihash_input_and_submissions(core, node_factory):  # noqa: F811
    node, addr = _eq_node(node_factory)
    c = client(node)
    tpl = c.getblocktemplate({"rules": ["segwit"]})
    assert "pprpcheader" not in tpl and tpl["version"] & core.EQUIHASH_VERSION_BIT
    eq = tpl["equihash"]
    assert (eq["n"], eq["k"], eq["personalization"], eq["solution_bytes"]) == (200, 9, "ZcashPoW", 1344)
    prefix = bytes.fromhex(eq["input"])
    assert len(prefix) == 80 and prefix[:4] == tpl["version"].to_bytes(4, "little")
    nonce256, sol = _solve_for_target(core, prefix, int(tpl["target"], 16))
    with pytest.raises(RuntimeError):
        c.equihashsubmit(eq["input"], nonce256.hex(), bytes(1344).hex())  # not a solution
    assert c.equihashsubmit(eq["input"], nonce256.hex(), sol.hex()) is True
    assert c.getblockcount() == 1
    # a full extended block through submitblock (what a Zcash-style miner sends)
    tpl2 = c.getblocktemplate({"rules": ["segwit"]})
    act = node.params.kawpow_activation_time
    blk = core.Block.deserialize(node.equihash_templates[tpl2["equihash"]["input"]].block.serialize(act), act)
    n2, s2 = _solve_for_target(core, bytes.fromhex(tpl2["equihash"]["input"]), int(tpl2["target"], 16), 1000)
    hdr = blk.header
    hdr.nonce256, hdr.solution = n2, s2
    blk.header = hdr
    assert c.submitblock(blk.serialize(act).hex()) is None
    assert c.getblockcount() == 2 and c.getbestblockhash() == core.u256_hex(hdr.equihash_hash(act))


def test_gloo_world2_mines_equihash(tmp_path, core):
    # 1 in 8 solutions is a share (target bits 3): a block every ~4 nonces per rank, so the CPU
    # golden solver (~2 s per nonce) finds both blocks well inside the deadline (at the default 7
    # bits the expected ~160 s made the test a coin toss against its 240 s limit)
    codes, outs, report = _run_world(tmp_path, 2, blocks=1, timeout_s=60.0,
                                     extra_env={"NODEXA_TEST_EQUIHASH": "1", "NODEXA_TEST_TARGET_BITS": "3"})
    assert codes == [0, 0], "\n".join(outs)
    rep = json.load(open(report))
    assert rep["height"] == 2 and rep["equihash_blocks"] == 2 and rep["stats"]["bad_shares"] == 0
    assert rep["coinbase"] == [["51"], ["52"]]
    assert all(int(v) > 0 for v in rep["rank_hashes"].values())  # both ranks found solutions
    assert [g["algo"] for g in rep["gpus_last"]] == ["equihash", "equihash"]


def test_remote_miner_mines_equihash(core, node_factory):  # noqa: F811
    from nodexa_chain_core_amd.miner.remote import RemoteMiner
    from nodexa_chain_core_amd.miner.service import make_rank_device

    node, addr = _eq_node(node_factory)
    c = client(node)
    m = RemoteMiner(c, make_rank_device(True), window=1, rank=1)
    stats = m.run(max_blocks=2, max_seconds=200)
    assert stats["accepted"] == 2 and stats["rejected"] == 0 and c.getblockcount() == 2
    hdr = core.Block.deserialize(bytes.fromhex(c.getblock(c.getbestblockhash(), 0)),
                                 node.params.kawpow_activation_time).header
    assert hdr.is_equihash() and int.from_bytes(hdr.nonce256[:8], "little") >> 56 == 1  # rank 1's nonce range


def test_bare_equihash_device_serves_equihash_windows(core):
    """A MiningService built on a bare Equihash device (bench.py's Equihash loop) sends the Equihash
    windows to THAT device -- not to a host golden solver made on first use -- and a KawPow packet
    on such a rank is a device fault, not a silent CPU search."""
    from nodexa_chain_core_amd.miner.equihash_search import EquihashCpuDevice
    from nodexa_chain_core_amd.miner.search import ALGO_EQUIHASH, ALGO_KAWPOW, DeviceFault, Work, as_rank_device

    dev = EquihashCpuDevice(window=3)
    rd = as_rank_device(dev)
    eq = Work(bytes(80), b"\xff" * 32, 1, 1, 0, 0, ALGO_EQUIHASH)
    assert rd.equihash is dev and rd.dev_for(eq) is dev and rd.window_for(eq, 16) == 3
    assert rd.name == dev.name and rd.resident_epochs() == []
    with pytest.raises(DeviceFault):
        rd.window_for(Work(bytes(32), b"\xff" * 32, 1, 1, 0, 0, ALGO_KAWPOW), 16)
