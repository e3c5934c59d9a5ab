"""Block template transaction selection by ancestor-package fee rate (addPackageTxs,
/root/reference/src/miner.cpp:380-500): a high-fee child pulls its low-fee parent in ahead of an
unrelated medium-fee transaction (CPFP), prioritisetransaction deltas count, and -blockmintxfee
ends selection."""
from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import spend


def _coins(c, n):
    w = c.getnewaddress()
    c.generatetoaddress(100 + n, w)
    coins = sorted((u for u in c.listunspent() if u["spendable"]), key=lambda u: (u["amount"], u["txid"]))
    assert len(coins) >= n
    return coins[-n:]


def _template_txids(c):
    return [t["txid"] for t in c.getblocktemplate()["transactions"]]


def test_child_pays_for_parent(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    u1, u2 = _coins(c, 2)
    dest = c.getnewaddress()
    # A: parent at the relay floor; C: unrelated, 5x A's rate; B: A's child paying 50x
    a = c.sendrawtransaction(spend(c, u1["txid"], u1["vout"], u1["amount"], dest, 10.0, fee=0.01))
    cc = c.sendrawtransaction(spend(c, u2["txid"], u2["vout"], u2["amount"], dest, 10.0, fee=0.05))
    b = c.sendrawtransaction(spend(c, a, 0, 10.0, c.getnewaddress(), 9.0, fee=0.5))
    assert _template_txids(c) == [a, b, cc]
    # prioritisetransaction: C's modified fee now beats the A+B package
    c.prioritisetransaction(cc, 0, 200_000_000)
    assert _template_txids(c) == [cc, a, b]
    tpl = c.getblocktemplate()["transactions"]
    assert tpl[2]["depends"] == [2]  # B still follows its parent A


def test_blockmintxfee_cuts_selection(core, node_factory):  # noqa: F811
    node, _ = node_factory(("-blockmintxfee=0.2",))
    c = client(node)
    u1, u2 = _coins(c, 2)
    dest = c.getnewaddress()
    lo = c.sendrawtransaction(spend(c, u1["txid"], u1["vout"], u1["amount"], dest, 10.0, fee=0.01))
    hi = c.sendrawtransaction(spend(c, u2["txid"], u2["vout"], u2["amount"], dest, 10.0, fee=0.1))
    txids = _template_txids(c)
    assert hi in txids and lo not in txids
