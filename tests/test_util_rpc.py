"""Utility RPCs: signed messages (signmessage / signmessagewithprivkey / verifymessage), multisig
(createmultisig, addmultisigaddress, partial signing through signrawtransaction with redeemScript,
combinerawtransaction) on a regtest node (src/rpc/misc.cpp, src/rpc/rawtransaction.cpp)."""
import os

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import fund, mature_coin, spend


def test_signed_messages(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    addr = c.getnewaddress()
    sig = c.signmessage(addr, "hello clore")
    assert c.verifymessage(addr, sig, "hello clore")
    assert not c.verifymessage(addr, sig, "hello clore!")
    wif = c.dumpprivkey(addr)
    assert c.verifymessage(addr, c.signmessagewithprivkey(wif, "other"), "other")
    assert not c.verifymessage(c.getnewaddress(), sig, "hello clore")
    with pytest.raises(RuntimeError, match="Malformed base64"):
        c.verifymessage(addr, "***", "x")


def test_multisig_partial_sign_and_combine(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    fund(c)
    secrets = []
    while len(secrets) < 3:
        k = os.urandom(32)
        if core.secp_seckey_valid(k):
            secrets.append(k)
    pubs = [core.secp_pubkey_create(k, True).hex() for k in secrets]
    wifs = [node.wallet.encode_wif(k) for k in secrets]
    ms = c.createmultisig(2, pubs)
    assert ms["redeemScript"].startswith("52") and ms["redeemScript"].endswith("53ae")
    with pytest.raises(RuntimeError, match="not enough keys"):
        c.createmultisig(4, pubs)
    u = mature_coin(c)
    fund_tx = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], ms["address"], 5.0))
    c.generatetoaddress(1, c.getnewaddress())
    out = c.gettxout(fund_tx, 0)
    assert out["value"] == 5.0
    raw = c.createrawtransaction([{"txid": fund_tx, "vout": 0}], {c.getnewaddress(): 4.99})
    prev = [{"txid": fund_tx, "vout": 0, "scriptPubKey": out["scriptPubKey"]["hex"], "redeemScript": ms["redeemScript"],
             "amount": 5.0}]
    a = c.signrawtransaction(raw, prev, [wifs[0]])
    b = c.signrawtransaction(raw, prev, [wifs[2]])
    assert not a["complete"] and not b["complete"]
    with pytest.raises(RuntimeError):
        c.sendrawtransaction(a["hex"])
    both = c.combinerawtransaction([a["hex"], b["hex"]])
    txid = c.sendrawtransaction(both)
    # signing on top of a partial copy completes it too
    assert c.signrawtransaction(a["hex"], prev, [wifs[1]])["complete"]
    c.generatetoaddress(1, c.getnewaddress())
    assert c.getrawtransaction(txid, True)["confirmations"] == 1
    # addmultisigaddress: the wallet remembers the script and signs with its own keys
    k1, k2 = c.getnewaddress(), c.getnewaddress()
    addr = c.addmultisigaddress(2, [k1, k2])
    assert addr == c.createmultisig(2, [k1, k2])["address"]
