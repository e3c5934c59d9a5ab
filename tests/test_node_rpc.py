"""End-to-end node on regtest (CPU PoW backend): JSON-RPC server + client,
KawPow mining through generate / getblocktemplate+pprpcsb / submitblock,
blk-file persistence and reload. Mirrors the reference's functional tests
(test/functional: mining_basic, mining_getblocktemplate_longpoll, rpc_*)."""
import json
import os
import struct
import threading

import pytest


# the engine's override that makes every mined regtest block KawPow (genesis time + 1); without it
# regtest keeps the reference's activation (3582830167) and mines X16RV2
KAWPOW_REGTEST = "-kawpowactivationtime=1524179367"


@pytest.fixture()
def node_factory(core, tmp_path):
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.utils.config import ArgsManager

    nodes = []

    def make(extra=(), kawpow=True):
        """kawpow=True: the KawPow-regtest override (every mined block KawPow); False: the
        reference's default regtest (X16RV2 until 2083)."""
        addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
        args = ArgsManager()
        flags = [KAWPOW_REGTEST] if kawpow else []
        args.parse_parameters(["-regtest", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                               f"-miningaddress={addr}", "-printtoconsole=0", *flags, *extra])
        n = Node(args)
        n.start()
        nodes.append(n)
        return n, addr

    yield make
    for n in nodes:
        n.stop()


def client(node):
    from nodexa_chain_core_amd.rpc.client import RPCClient

    return RPCClient("127.0.0.1", node.rpc.port, "u", "p")


def test_generate_and_query(core, node_factory):
    node, addr = node_factory()
    c = client(node)
    assert c.getblockcount() == 0
    hashes = c.generatetoaddress(3, addr)
    assert len(hashes) == 3 and c.getblockcount() == 3
    assert c.getbestblockhash() == hashes[-1]
    assert c.getblockhash(3) == hashes[-1]
    blk = c.getblock(hashes[0])
    assert blk["height"] == 1 and blk["nTx"] == 1 and blk["confirmations"] == 3
    assert {"headerhash", "mixhash", "nonce64"} <= set(blk)  # KawPow fields (src/rpc/blockchain.cpp:254-256)
    hdr = c.getblockheader(hashes[1])
    assert hdr["previousblockhash"] == hashes[0] and hdr["nextblockhash"] == hashes[2]
    raw = bytes.fromhex(c.getblock(hashes[0], 0))
    p = node.params
    b = core.Block.deserialize(raw, p.kawpow_activation_time)
    # coinbase: miner + community-autonomous output + witness commitment
    cb = b.vtx[0]
    sub = core.block_subsidy(1)
    assert cb.vout[1].value == sub * p.community_autonomous_pct // 100
    assert core.script_to_address(cb.vout[1].script_pubkey, p.pubkey_prefix, p.script_prefix) == \
        p.community_autonomous_address
    # getkawpowhash agrees with the stored header
    res = c.getkawpowhash(blk["headerhash"], blk["mixhash"], "%016x" % blk["nonce64"], 1, "7f" + "ff" * 31)
    assert res["result"] == "true" and res["meets_target"] == "true" and res["digest"] == hashes[0]
    info = c.getmininginfo()
    assert info["blocks"] == 3 and info["chain"] == "regtest"
    assert c.submitblock(raw.hex()) == "duplicate"
    assert c.call("verifychain", 4, 3) is True


def test_gbt_pprpcsb_roundtrip(core, node_factory):
    node, addr = node_factory()
    c = client(node)
    tpl = c.getblocktemplate({"rules": ["segwit"]})
    for k in ("previousblockhash", "coinbasevalue", "CommunityAutonomousAddress", "CommunityAutonomousValue", "target",
              "bits", "height", "pprpcheader", "pprpcepoch", "default_witness_commitment", "longpollid"):
        assert k in tpl, k
    # an external miner: search nNonce64 for the template's KawPow header hash
    header_hash = bytes.fromhex(tpl["pprpcheader"])
    boundary = bytes.fromhex(tpl["target"])
    ctx = core.get_epoch_context(tpl["pprpcepoch"])
    ok, nonce, fin, mix = core.kawpow_search_light(ctx, tpl["height"], header_hash, boundary, 0, 1000)
    assert ok
    assert c.pprpcsb(tpl["pprpcheader"], mix.hex(), "%016x" % nonce) is True
    assert c.getblockcount() == 1
    with pytest.raises(RuntimeError, match="not found"):
        c.pprpcsb("00" * 32, mix.hex(), "%016x" % nonce)


def test_gbt_depends_and_sigops(core, node_factory):
    """getblocktemplate `depends` lists in-template parents by 1-based position and `sigops` is the
    transaction's sigop cost (src/rpc/mining.cpp:585-617); pool software must not assume []/0."""
    from wallet_util import fund, mature_coin, spend

    node, addr = node_factory()
    c = client(node)
    w = fund(c, 101)
    u = mature_coin(c)
    parent = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], w, 5.0))
    child = c.sendrawtransaction(spend(c, parent, 0, 5.0, w, 4.0))
    tpl = c.getblocktemplate({"rules": ["segwit"]})
    txs = {t["txid"]: (i + 1, t) for i, t in enumerate(tpl["transactions"])}
    assert set(txs) == {parent, child}
    ppos, pent = txs[parent]
    cpos, cent = txs[child]
    assert ppos == 1 and cpos == 2
    assert pent["depends"] == [] and cent["depends"] == [1]
    # two P2PKH outputs (OP_CHECKSIG each) x WITNESS_SCALE_FACTOR; P2PKH inputs add nothing
    assert pent["sigops"] == cent["sigops"] == 8
    raw = bytes.fromhex(cent["data"])
    assert cent["sigops"] == core.tx_legacy_sigops(raw) * 4


def test_submitblock_rejects(core, node_factory):
    node, addr = node_factory()
    c = client(node)
    from nodexa_chain_core_amd.miner.assembler import BlockAssembler

    tpl = BlockAssembler(node.state).create_new_block(node.mining_script)
    blk = tpl.block
    act = node.params.kawpow_activation_time
    # wrong community amount -> bad-cb-community-autonomous-amount
    bad = core.Block.deserialize(blk.serialize(act), act)
    cb = bad.vtx[0]
    outs = list(cb.vout)
    outs[1] = core.TxOut(outs[1].value + 1, outs[1].script_pubkey)
    cb.vout = outs
    bad.vtx = [cb]
    h = bad.header
    h.merkle_root = bad.merkle_root()[0]
    ctx = core.get_epoch_context(0)
    for n in range(64):  # solve it (regtest target 2^255): the reward rule is checked at connection
        fin, mix = core.kawpow_hash(ctx, h.height, h.kawpow_header_hash()[::-1], n)
        if fin[0] < 0x80:
            h.nonce64, h.mix_hash = n, mix[::-1]
            break
    bad.header = h
    assert c.submitblock(bad.serialize(act).hex()) == "bad-cb-community-autonomous-amount"
    # merkle mismatch
    bad2 = core.Block.deserialize(blk.serialize(act), act)
    h = bad2.header
    h.merkle_root = bytes(32)
    bad2.header = h
    assert c.submitblock(bad2.serialize(act).hex()) == "bad-txnmrklroot"
    # unsolved header -> high-hash (regtest target is 2^255: pick a failing nonce)
    ctx = core.get_epoch_context(0)
    h = blk.header
    for n in range(64):
        h.nonce64 = n
        fin, mix = core.kawpow_hash(ctx, h.height, h.kawpow_header_hash()[::-1], n)
        if fin[0] >= 0x80:
            h.mix_hash = mix[::-1]
            break
    blk.header = h
    assert c.submitblock(blk.serialize(act).hex()) == "high-hash"


def test_restart_reloads_blocks(core, node_factory, tmp_path):
    node, addr = node_factory()
    c = client(node)
    hashes = c.generatetoaddress(2, addr)
    node.stop()
    # blk file framing: magic, size, block (src/validation.cpp:1275-1294)
    raw = open(os.path.join(str(tmp_path), "regtest", "blocks", "blk00000.dat"), "rb").read()
    assert raw[:4] == b"DROW"
    n2, _ = node_factory()
    c2 = client(n2)
    assert c2.getblockcount() == 2 and c2.getbestblockhash() == hashes[-1]


def test_rpc_protocol_errors(node_factory):
    node, _ = node_factory()
    c = client(node)
    status, rep = c.call_raw({"method": "nosuchmethod", "params": [], "id": 7})
    assert status == 404 and rep["error"]["code"] == -32601 and rep["id"] == 7
    rep = c.batch([("getblockcount", []), ("getblockhash", [99])])
    assert rep[0]["result"] == 0 and rep[1]["error"]["code"] == -8
    from nodexa_chain_core_amd.rpc.client import RPCClient

    bad = RPCClient("127.0.0.1", node.rpc.port, "u", "wrong")
    with pytest.raises(PermissionError):
        bad.getblockcount()
    assert "getblocktemplate" in c.help()
    # named parameters
    status, rep = c.call_raw({"method": "getblockhash", "params": {"height": 0}, "id": 1})
    assert rep["result"] == c.getbestblockhash()


def test_cli_main(node_factory, capsys, tmp_path):
    node, _ = node_factory()
    from nodexa_chain_core_amd.rpc.client import main

    rc = main(["-regtest", f"-datadir={tmp_path}", f"-rpcport={node.rpc.port}", "-rpcuser=u", "-rpcpassword=p",
               "getblockcount"])
    assert rc == 0 and capsys.readouterr().out.strip() == "0"


def test_generate_x16rv2_reference_default(core, node_factory):
    """BASELINE config 1 with the reference's own regtest params, which are this engine's default
    regtest (no flag): KawPow activation in 2083 (src/chainparams.cpp:566-570), so `generate`
    hashes 80-byte X16RV2 headers and bumps the 32-bit nNonce (src/rpc/mining.cpp:117-173)."""
    node, addr = node_factory(kawpow=False)
    assert node.params.kawpow_activation_time == 3582830167
    c = client(node)
    hashes = c.generatetoaddress(2, addr)
    assert c.getblockcount() == 2
    p = node.params
    raw = bytes.fromhex(c.getblock(hashes[1], 0))
    b = core.Block.deserialize(raw, p.kawpow_activation_time)
    h = b.header
    assert h.time < p.kawpow_activation_time and h.time >= p.x16rv2_activation_time
    assert len(h.legacy80()) == 80
    got = core.x16rv2(h.legacy80(), h.prev)
    assert core.u256_hex(got) == hashes[1]
    target, _, _ = core.set_compact(h.bits)
    assert int.from_bytes(got, "little") <= target
    # batch verifier handles legacy headers too (CPU X16RV2), and rejects a bumped nonce
    from nodexa_chain_core_amd.models.verify import verify_headers

    hdrs = [core.Block.deserialize(bytes.fromhex(c.getblock(x, 0)), p.kawpow_activation_time).header for x in hashes]
    res = verify_headers(p, hdrs)
    assert all(r["valid"] for r in res) and [r["hash"] for r in res] == hashes
    bad = hdrs[0]
    for k in range(1, 64):  # find a nonce that misses the regtest target (~1/2 of nonces do)
        bad.nonce = (bad.nonce + 1) & 0xFFFFFFFF
        if not verify_headers(p, [bad])[0]["valid"]:
            break
    assert verify_headers(p, [bad])[0]["reason"] == "high-hash"


def test_mempool_rpcs_and_rest(core, node_factory):
    node, addr = node_factory()
    c = client(node)
    hashes = c.generatetoaddress(2, addr)
    assert c.getmempoolinfo()["size"] == 0
    code, _, body = node.rest("/rest/mempool/info.json")
    assert code == 200 and json.loads(body)["size"] == 0
    code, _, body = node.rest("/rest/blockhashbyheight/2.json")
    assert code == 200 and json.loads(body)["blockhash"] == hashes[1]
    assert node.rest("/rest/blockhashbyheight/99.json")[0] == 404
    blk = c.getblock(hashes[0])
    cb = blk["tx"][0]
    raw = c.getrawtransaction(cb, False, hashes[0])
    assert c.decoderawtransaction(raw)["txid"] == cb
    assert c.getrawtransaction(cb, True, hashes[0])["blockhash"] == hashes[0]


def test_regtest_kawpow_is_an_override(core, node_factory):
    """The reference's explicit value and the engine default agree; only the override flag moves the
    activation, and a KawPow-regtest `generate` makes 120-byte KawPow headers."""
    from nodexa_chain_core_amd.chain.state import REGTEST_KAWPOW_FROM_GENESIS, make_params

    assert make_params("regtest").kawpow_activation_time == core.make_chain_params("regtest").kawpow_activation_time \
        == 3582830167
    assert make_params("regtest", REGTEST_KAWPOW_FROM_GENESIS).kawpow_activation_time == 1524179367
    node, addr = node_factory()
    c = client(node)
    h = c.generatetoaddress(1, addr)[0]
    raw = bytes.fromhex(c.getblockheader(h, False))
    assert len(raw) == 120 and core.BlockHeader.deserialize(raw, node.params.kawpow_activation_time).height == 1
