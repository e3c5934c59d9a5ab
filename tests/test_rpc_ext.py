"""The extended RPC table (rpc/methods_ext.py) on a regtest node with the CPU PoW backend.

Mirrors the reference's functional tests for these commands: rpc_blockchain.py
(getchaintxstats, waitforblockheight), mempool_persist.py (savemempool / -persistmempool),
mempool_packages.py (ancestors / descendants), rpc_txoutproof.py, rpc_rawtransaction.py
(createrawtransaction / decodescript), mempool_accept.py (testmempoolaccept),
p2p_disconnect_ban.py (setban / listbanned / clearbanned / disconnectnode) and
rpc_net.py (getnettotals, setnetworkactive)."""
import os

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import fund, mature_coin, spend


def _rpc_error(fn, *a):
    with pytest.raises(RuntimeError) as e:
        fn(*a)
    return str(e.value)


def _tx(c, addr, prev_txid, vout=0, amount=1.0):
    return c.createrawtransaction([{"txid": prev_txid, "vout": vout}], {addr: amount})


def test_control_and_hidden(core, node_factory):  # noqa: F811
    node, addr = node_factory()
    c = client(node)
    c.generatetoaddress(3, addr)
    info = c.getinfo()
    assert info["blocks"] == 3 and "deprecation-warning" in info and info["testnet"] is False
    assert c.echo("a", 1, [2]) == ["a", 1, [2]]
    c.setmocktime(2_000_000_000)
    assert node.state.adjusted_time() == 2_000_000_000
    c.setmocktime(0)
    assert "not in prune mode" in _rpc_error(c.pruneblockchain, 1)
    assert c.waitforblockheight(2, 10)["height"] == 3
    assert c.waitforblock(c.getbestblockhash(), 10)["height"] == 3
    est = c.estimatesmartfee(6)
    assert est["errors"] and est["blocks"] == 0  # clamped to the (empty) usable history
    assert "deprecated" in _rpc_error(c.estimatefee, 6)
    assert "fail" in c.estimaterawfee(6)["short"]


def test_mempool_packages_persist_and_proofs(core, node_factory):  # noqa: F811
    node, addr = node_factory()
    c = client(node)
    fund(c)
    u = mature_coin(c)
    parent = spend(c, u["txid"], u["vout"], u["amount"], addr, 1.0)
    dec = c.decoderawtransaction(parent)
    assert dec["vout"][0]["valueSat"] == 100_000_000
    assert c.testmempoolaccept([parent]) == [{"txid": dec["txid"], "allowed": True}]
    ptxid = c.sendrawtransaction(parent)
    res = c.testmempoolaccept([parent])[0]
    assert not res["allowed"] and "txn-already-in-mempool" in res["reject-reason"]
    bad = c.createrawtransaction([{"txid": "22" * 32, "vout": 0}, {"txid": "22" * 32, "vout": 0}], {addr: 1})
    assert "bad-txns-inputs-duplicate" in c.testmempoolaccept([bad])[0]["reject-reason"]
    assert "missing-inputs" in c.testmempoolaccept([_tx(c, addr, "33" * 32)])[0]["reject-reason"]
    change = dec["vout"][1]["value"]
    child = spend(c, ptxid, 1, change, addr, 0.5)
    ctxid = c.sendrawtransaction(child)
    assert c.getmempoolancestors(ctxid) == [ptxid]
    assert c.getmempooldescendants(ptxid) == [ctxid]
    e = c.getmempoolentry(ctxid)
    assert e["ancestorcount"] == 2 and e["depends"] == [ptxid] and e["descendantcount"] == 1
    assert list(c.getmempooldescendants(ptxid, True)) == [ctxid]
    # a second spend of the parent's change conflicts with the child
    assert "txn-mempool-conflict" in c.testmempoolaccept([spend(c, ptxid, 1, change, addr, 0.25)])[0]["reject-reason"]
    # savemempool + restart (-persistmempool default on): both re-enter through AcceptToMemoryPool
    c.savemempool()
    assert os.path.exists(os.path.join(node.datadir, "mempool.dat"))
    node.stop()
    node, _ = node_factory()
    c = client(node)
    assert sorted(c.getrawmempool()) == sorted([ptxid, ctxid])
    # mine them, then prove inclusion (BIP37 partial merkle tree)
    h = c.generatetoaddress(1, addr)[0]
    assert c.getmempoolinfo()["size"] == 0
    blk = c.getblock(h)
    assert ptxid in blk["tx"] and ctxid in blk["tx"]
    proof = c.gettxoutproof([ctxid])
    assert c.verifytxoutproof(proof) == [ctxid]
    proof2 = c.gettxoutproof([ptxid, ctxid], h)
    assert sorted(c.verifytxoutproof(proof2)) == sorted([ptxid, ctxid])
    tampered = proof[:-2] + ("00" if proof[-2:] != "00" else "01")
    with pytest.raises(RuntimeError):
        assert c.verifytxoutproof(tampered) == [ctxid]
    # chain tx stats: genesis + one coinbase per block + the 2 spends
    height = c.getblockcount()
    stats = c.getchaintxstats()
    assert stats["txcount"] == 1 + height + 2
    assert c.decodeblock(c.getblock(h, 0))["hash"] == h
    # clearmempool
    u = mature_coin(c)
    c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], addr, 1.0))
    c.clearmempool()
    assert c.getmempoolinfo()["size"] == 0
    # getblockhashes over the whole time range returns the active chain (minus genesis time filter)
    hs = c.getblockhashes(2**31 - 1, 0)
    assert h in hs and len(hs) == height + 1


def test_decodescript(core, node_factory):  # noqa: F811
    node, addr = node_factory()
    c = client(node)
    spk = core.address_to_script(addr, node.params.pubkey_prefix, node.params.script_prefix)
    d = c.decodescript(spk.hex())
    assert d["type"] == "pubkeyhash" and d["addresses"] == [addr]
    assert d["asm"] == f"OP_DUP OP_HASH160 {spk[3:23].hex()} OP_EQUALVERIFY OP_CHECKSIG"
    assert d["p2sh"]
    assert c.decodescript("6a0401020304")["asm"] == "OP_RETURN 67305985"
    assert c.decodescript("52ae")["type"] == "nonstandard"


def test_network_rpcs(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    assert "-31" in _rpc_error(c.listbanned)
    node.stop()
    node2, _ = node_factory(("-listen", "-port=0"))
    c2 = client(node2)
    c2.setban("10.1.2.3", "add", 3600)
    assert [b["address"] for b in c2.listbanned()] == ["10.1.2.3"]
    assert "-23" in _rpc_error(c2.setban, "10.1.2.3", "add")
    c2.setban("10.1.2.3", "remove")
    assert c2.listbanned() == []
    c2.setban("10.9.9.9", "add")
    c2.clearbanned()
    assert c2.listbanned() == []
    assert "-30" in _rpc_error(c2.setban, "not-an-ip", "add")
    tot = c2.getnettotals()
    assert {"totalbytesrecv", "totalbytessent", "timemillis", "uploadtarget"} <= set(tot)
    assert c2.getaddednodeinfo() == []
    assert "-24" in _rpc_error(c2.addnode, "127.0.0.1:1", "remove")
    assert "-29" in _rpc_error(c2.disconnectnode, "127.0.0.1:1")
    assert c2.setnetworkactive(False) is False
    assert c2.setnetworkactive(True) is True


def test_rest_block_tx_headers(core, node_factory):  # noqa: F811
    import json

    node, addr = node_factory()
    c = client(node)
    hashes = c.generatetoaddress(3, addr)
    code, _, body = node.rest(f"/rest/block/{hashes[1]}.json")
    blk = json.loads(body)
    assert code == 200 and blk["hash"] == hashes[1] and isinstance(blk["tx"][0], dict)
    code, _, body = node.rest(f"/rest/block/notxdetails/{hashes[1]}.json")
    assert code == 200 and isinstance(json.loads(body)["tx"][0], str)
    code, _, body = node.rest(f"/rest/block/notxdetails/{hashes[1]}.hex")
    assert body.decode() == c.getblock(hashes[1], 0)
    code, _, body = node.rest(f"/rest/headers/2/{hashes[0]}.json")
    assert [h["hash"] for h in json.loads(body)] == hashes[:2]
    assert node.rest(f"/rest/headers/0/{hashes[0]}.json")[0] == 400
    fund(c)
    u = mature_coin(c)
    txid = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], addr, 1.0))
    code, _, body = node.rest(f"/rest/tx/{txid}.json")
    assert code == 200 and json.loads(body)["txid"] == txid
    assert node.rest(f"/rest/tx/{txid}.hex")[2].decode() == c.getrawtransaction(txid)
    assert node.rest(f"/rest/tx/{'55' * 32}.json")[0] == 404


def test_bip9_versionbits_regtest(core, node_factory):  # noqa: F811
    """BIP9 on regtest (window 144 / threshold 108; transfer_script 288 / 208; coinbase 500 / 400):
    deployments start after the first period, lock in after a signalling period and activate one
    period later (feature_versionbits / rpc_blockchain bip9_softforks in the reference)."""
    node, addr = node_factory()
    c = client(node)
    c.generatetoaddress(433, addr)
    forks = c.getblockchaininfo()["bip9_softforks"]
    assert forks["assets"]["status"] == "active" and forks["assets"]["since"] == 432
    assert forks["testdummy"]["status"] == "active"
    ts = forks["transfer_script"]
    assert ts["status"] == "started" and ts["since"] == 288 and ts["bit"] == 8
    assert ts["statistics"]["period"] == 288 and ts["statistics"]["elapsed"] == 433 - 287
    assert ts["statistics"]["count"] == ts["statistics"]["elapsed"] and ts["statistics"]["possible"]
    assert forks["coinbase"]["status"] == "defined"
    blk = c.getblock(c.getblockhash(200))
    assert blk["version"] & 0xE0000000 == 0x20000000 and blk["version"] & (1 << 6)  # signalled assets
    tpl = c.getblocktemplate()
    assert set(tpl["rules"]) == {"testdummy", "assets", "messaging_restricted", "enforce_value"}
    assert tpl["vbavailable"] == {"transfer_script": 8} and tpl["vbrequired"] == 0
    assert tpl["version"] == 0x30000000 | (1 << 8)


def test_stopatheight_and_reorg_flags(core, node_factory):  # noqa: F811
    node, addr = node_factory(("-stopatheight=3", "-maxreorg=7", "-minreorgpeers=1"))
    c = client(node)
    assert node.params.max_reorg_depth == 7 and node.params.min_reorg_peers == 1
    c.generatetoaddress(2, addr)
    assert not node.shutdown_requested()
    c.generatetoaddress(1, addr)
    assert node.shutdown_requested()
    # armed only with enough peers and a fresh tip
    assert node.state.arm_reorg_guard(1) and node.state.chain.max_reorg_depth == 7
    assert not node.state.arm_reorg_guard(0) and node.state.chain.max_reorg_depth == 0
