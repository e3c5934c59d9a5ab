"""-txindex / -addressindex / -spentindex / -timestampindex through their RPCs and
REST: address deltas, balances, unspent outputs and txids, spent info, block deltas, timestamp
lookups and getrawtransaction without a block hash; reorgs unwind every index; a restart keeps
them; REST getutxos."""
import json

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import fund, mature_coin, spend

INDEX_ARGS = ("-txindex", "-addressindex", "-spentindex", "-timestampindex")


def test_address_and_spent_indexes(core, node_factory):  # noqa: F811
    node, _ = node_factory(INDEX_ARGS)
    c = client(node)
    w = fund(c)
    dest = c.getnewaddress()
    u = mature_coin(c)
    txid = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], dest, 12.5))
    # mempool view first
    pool = c.getaddressmempool({"addresses": [dest]})
    assert [(r["txid"], r["satoshis"]) for r in pool] == [(txid, 1_250_000_000)]
    h = c.generatetoaddress(1, w)[0]
    height = c.getblockcount()
    # deltas / balance / utxos / txids of the receiving address
    d = c.getaddressdeltas({"addresses": [dest]})
    assert [(x["txid"], x["satoshis"], x["height"], x["address"]) for x in d] == [(txid, 1_250_000_000, height, dest)]
    assert c.getaddressbalance({"addresses": [dest]}) == {"balance": 1_250_000_000, "received": 1_250_000_000}
    utxos = c.getaddressutxos({"addresses": [dest]})
    assert [(x["txid"], x["outputIndex"], x["satoshis"]) for x in utxos] == [(txid, 0, 1_250_000_000)]
    assert c.getaddresstxids({"addresses": [dest]}) == [txid]
    # the spent coinbase output: spent info, and a negative delta for the mining address
    info = c.getspentinfo({"txid": u["txid"], "index": u["vout"]})
    assert info == {"txid": txid, "index": 0, "height": height}
    mined = c.getaddressdeltas({"addresses": [w]})
    assert any(x["txid"] == txid and x["satoshis"] == -round(u["amount"] * 1e8) for x in mined)
    ranged = c.getaddressdeltas({"addresses": [w], "start": 1, "end": 2, "chainInfo": True})
    assert ranged["start"]["height"] == 1 and all(1 <= x["height"] <= 2 for x in ranged["deltas"])
    # block deltas and the indexes behind getrawtransaction / getblockhashes / gettxoutproof
    bd = c.getblockdeltas(h)
    assert bd["height"] == height and bd["deltas"][1]["txid"] == txid
    assert bd["deltas"][1]["inputs"][0]["prevtxid"] == u["txid"]
    assert c.getrawtransaction(txid, True)["blockhash"] == h
    blk = c.getblock(h)
    assert h in c.getblockhashes(blk["time"] + 1, blk["time"])
    assert c.verifytxoutproof(c.gettxoutproof([txid])) == [txid]
    # spend the indexed output: its utxo entry goes, a spending delta appears
    tx2 = c.sendrawtransaction(spend(c, txid, 0, 12.5, w, 10))
    c.generatetoaddress(1, w)
    assert c.getaddressutxos({"addresses": [dest]}) == []
    assert c.getaddressbalance({"addresses": [dest]})["balance"] == 0
    assert c.getaddresstxids({"addresses": [dest]}) == [txid, tx2]
    # reorg: disconnecting both blocks unwinds every index
    c.invalidateblock(h)
    assert c.getaddressdeltas({"addresses": [dest]}) == []
    assert c.getaddressutxos({"addresses": [dest]}) == []
    try:
        c.getspentinfo({"txid": u["txid"], "index": u["vout"]})
        raise AssertionError("spent info survived the disconnect")
    except RuntimeError as e:
        assert "Unable to get spent info" in str(e)
    assert h not in c.getblockhashes(blk["time"] + 1, blk["time"])
    c.reconsiderblock(h)
    assert c.getaddressbalance({"addresses": [dest]}) == {"balance": 0, "received": 1_250_000_000}
    # restart keeps the indexes
    node.stop()
    node, _ = node_factory(INDEX_ARGS)
    c = client(node)
    assert c.getaddresstxids({"addresses": [dest]}) == [txid, tx2]
    assert c.getspentinfo({"txid": txid, "index": 0})["txid"] == tx2


def test_rest_getutxos_and_tx(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    fund(c)
    u = mature_coin(c)
    code, _, body = node.rest(f"/rest/getutxos/{u['txid']}-{u['vout']}/{'00' * 32}-0.json")
    res = json.loads(body)
    assert code == 200 and res["bitmap"] == "10" and len(res["utxos"]) == 1
    assert res["utxos"][0]["value"] == u["amount"]
    txid = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], c.getnewaddress(), 1.0))
    # spent in the mempool: still unspent on chain, gone in the mempool view, whose new outputs count
    assert json.loads(node.rest(f"/rest/getutxos/{u['txid']}-{u['vout']}.json")[2])["bitmap"] == "1"
    res = json.loads(node.rest(f"/rest/getutxos/checkmempool/{u['txid']}-{u['vout']}/{txid}-0.json")[2])
    assert res["bitmap"] == "01" and res["utxos"][0]["height"] == 0x7FFFFFFF
    code, _, raw = node.rest(f"/rest/getutxos/{u['txid']}-{u['vout']}.bin")
    assert code == 200 and raw[36:38] == b"\x01\x01" and raw[38] == 1  # bitmap [1], one coin
    assert node.rest("/rest/getutxos/" + "/".join([f"{'11' * 32}-{i}" for i in range(16)]) + ".json")[0] == 400
    # /rest/tx finds a confirmed transaction through its unspent outputs (GetTransaction)
    h = c.generatetoaddress(1, c.getnewaddress())[0]
    code, _, body = node.rest(f"/rest/tx/{txid}.json")
    assert code == 200 and json.loads(body)["blockhash"] == h
