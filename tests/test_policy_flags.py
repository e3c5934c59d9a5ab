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


def test_safe_mode(core, node_factory, tmp_path):  # noqa: F811
    """-testsafemode: the reference's ObserveSafeMode RPCs refuse with RPC_FORBIDDEN_BY_SAFE_MODE,
    the warning shows in getblockchaininfo / getnetworkinfo / getmininginfo; -disablesafemode
    overrides it; other RPCs are unaffected."""
    node, _ = node_factory(("-testsafemode",))
    c = client(node)
    with pytest.raises(RuntimeError, match=r"RPC error -2: Safe mode: testsafemode enabled"):
        c.getbalance()
    assert c.getblockchaininfo()["warnings"] == "testsafemode enabled"
    assert c.getmininginfo()["warnings"] == "testsafemode enabled"
    assert c.getblockcount() == 0
    node.stop()
    node, _ = node_factory(("-testsafemode", "-disablesafemode"))
    assert client(node).getbalance() == 0


def test_dns_off_and_sysperms(core, node_factory, tmp_path):  # noqa: F811
    import os
    import stat

    node, _ = node_factory(("-listen=1", "-port=0", "-listenonion=0", "-dns=0"))
    with pytest.raises(ConnectionError, match="DNS lookups are disabled"):
        node.connman.connect("localhost", 1)
    # without -sysperms the node's files are private to its user (umask 077)
    mode = os.stat(os.path.join(node.datadir, "debug.log")).st_mode
    assert stat.S_IMODE(mode) & 0o077 == 0


def test_discardfee_drops_dust_change(core, node_factory):  # noqa: F811
    node, _ = node_factory(("-discardfee=0.0001",))
    c = client(node)
    fund(c)
    w = node.wallet
    assert w._change_discard_threshold() == (34 + 148) * 10_000 // 1000
    # selection is largest-first, so size the payments against the coin the wallet itself picks
    # for a payment of half the largest listed coin (that one input's value = outputs + fee)
    top = max(round(u["amount"] * 1e8) for u in c.listunspent())
    from nodexa_chain_core_amd.wallet.wallet import WalletError

    for _ in range(8):
        dest = core.address_to_script(c.getnewaddress(), node.params.pubkey_prefix, node.params.script_prefix)
        # a fixed 1 sat/B: a signature one byte longer or shorter moves the fee by 1 sat, not by
        # more than the dust margin (the node's own rate can be thousands of sat/B here)
        tx, fee = w.create_transaction([(dest, top // 2)], fee_rate=1000)
        assert len(tx.vout) == 2  # ordinary change
        if len(tx.vin) != 1:
            continue
        coin = sum(o.value for o in tx.vout) + fee
        amount = coin - fee - 1000  # would leave 1000 sat of change: dust at the discard rate
        try:
            tx2, fee2 = w.create_transaction([(dest, amount)], fee_rate=1000)
        except WalletError:
            # the second signature came out one byte longer than the first (DER length varies with
            # R and S): at this fee rate that byte costs more than the 1000 sat, so no change is
            # left at all; another destination gives other signatures
            continue
        assert len(tx2.vout) == 1 and fee2 == coin - amount, (len(tx2.vin), [o.value for o in tx2.vout], fee2, coin,
                                                               amount, fee)
        break
    else:
        raise AssertionError("no attempt left dust change to discard")


def test_walletrejectlongchains(core, node_factory):  # noqa: F811
    node, _ = node_factory(("-walletrejectlongchains", "-limitancestorcount=2"))
    c = client(node)
    fund(c)
    to = c.getnewaddress()
    c.sendtoaddress(to, 1.0)  # spends the one mature coin; its change is unconfirmed
    c.sendtoaddress(to, 1.0)  # spends that change (ancestors: 1)
    with pytest.raises(RuntimeError, match="too long of a mempool chain"):
        c.sendtoaddress(to, 1.0)
