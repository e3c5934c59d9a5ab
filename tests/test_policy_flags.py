"""-bytespersigop (sigop-adjusted virtual size, GetVirtualTransactionSize in
/root/reference/src/policy/policy.cpp) and -dbcache (the UTXO changes held between flushes,
/root/reference/src/init.cpp nCoinCacheUsage)."""
import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import fund, mature_coin


def _sigop_heavy_tx(c, fee: float) -> str:
    """A spend with an extra zero-value output of 20 OP_CHECKSIGs: 20 legacy sigops (cost 80)
    in a ~260-byte transaction."""
    u = mature_coin(c)
    outs = {c.getnewaddress(): round(u["amount"] - fee, 8), "data": "00"}
    raw = c.createrawtransaction([{"txid": u["txid"], "vout": u["vout"]}], outs)
    op_return = "0000000000000000" + "03" + "6a0100"
    assert op_return in raw
    raw = raw.replace(op_return, "0000000000000000" + "14" + "ac" * 20)
    signed = c.signrawtransaction(raw)
    assert signed["complete"]
    return signed["hex"]


@pytest.mark.parametrize("bps, accepted", [(None, False), (1, True)])
def test_bytespersigop_prices_sigops(core, node_factory, bps, accepted):  # noqa: F811
    extra = () if bps is None else (f"-bytespersigop={bps}",)
    node, _ = node_factory(extra)
    c = client(node)
    fund(c)
    # 0.003 covers the real size (~260 vB at the 0.01 / kvB relay floor) but not the
    # sigop-adjusted one at the default 20 bytes per sigop: 80 x 20 / 4 = 400 vB
    tx = _sigop_heavy_tx(c, 0.003)
    if accepted:
        txid = c.sendrawtransaction(tx)
        e = c.getmempoolentry(txid)
        assert e["size"] < 400
    else:
        with pytest.raises(RuntimeError, match="min relay fee not met"):
            c.sendrawtransaction(tx)


def test_dbcache_bounds_pending_utxo_changes(core, node_factory):  # noqa: F811
    node, addr = node_factory(("-dbcache=4",))
    st = node.state
    assert st.coins_cache_bytes == 4 << 20
    c = client(node)
    c.generatetoaddress(3, addr)
    assert st._since_flush == 3  # far below both the block interval and the cache bound
    st.coins_cache_bytes = 600   # a few pending coin changes: the next blocks flush
    c.generatetoaddress(6, addr)
    assert st._since_flush < 6
    assert c.gettxoutsetinfo()["height"] == 9
