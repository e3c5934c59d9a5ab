"""Wallet RPCs beyond the basic set: watch-only imports, BIP125 replacement and bumpfee, accounts
(move / sendfrom / getbalance "account"), sendfromaddress, getmasterkeyinfo, pruned-funds import,
and the relay-policy output rules (IsStandardTx) that mainnet applies."""
import hashlib

import pytest

from test_node_rpc import client
from test_p2p import _node
from test_wallet import BIP39_VECTORS
from wallet_util import fund


def _key(core, seed: bytes):
    secret = hashlib.sha256(seed).digest()
    pub = core.secp_pubkey_create(secret, True)
    return secret, pub, core.base58check_encode(bytes([42]) + core.hash160(pub))


def test_watch_only_imports(core, tmp_path):
    node = _node(core, tmp_path, "w", [])
    try:
        c = client(node)
        fund(c, 110)
        _, pub1, addr1 = _key(core, b"watch-1")
        _, pub2, addr2 = _key(core, b"watch-2")
        c.importaddress(addr1, "cold", False)
        c.importpubkey(pub2.hex(), "cold2", False)
        c.sendtoaddress(addr1, 5)
        c.sendtoaddress(addr2, 7)
        c.generatetoaddress(1, c.getnewaddress())
        rows = {u["address"]: u for u in c.listunspent() if u["address"] in (addr1, addr2)}
        assert rows[addr1]["spendable"] is False and rows[addr1]["solvable"] is False
        assert rows[addr2]["solvable"] is True and rows[addr2]["account"] == "cold2"
        mine = c.getbalance()
        assert c.getbalance("*", 1, True) == pytest.approx(mine + 12)
        assert c.validateaddress(addr1)["ismine"] is False
        wo = [e for e in c.listtransactions("*", 50, 0, True) if e.get("involvesWatchonly")]
        assert {e["address"] for e in wo if e["category"] == "receive"} == {addr1, addr2}
        assert not any(e.get("involvesWatchonly") for e in c.listtransactions("*", 50, 0, False))
        with pytest.raises(RuntimeError, match="already contains the private key"):
            c.importaddress(c.getnewaddress())
        # importmulti: a key (becomes spendable) and a watch-only script in one call
        secret3, _, addr3 = _key(core, b"multi-3")
        wif3 = core.base58check_encode(bytes([114]) + secret3 + b"\x01")
        _, _, addr4 = _key(core, b"multi-4")
        res = c.importmulti([{"scriptPubKey": {"address": addr3}, "timestamp": 0, "keys": [wif3]},
                             {"scriptPubKey": {"address": addr4}, "timestamp": 0, "label": "w4"},
                             {"scriptPubKey": {"address": addr4}}], {"rescan": False})
        assert [r["success"] for r in res] == [True, True, False]
        assert c.validateaddress(addr3)["ismine"] is True
        # addwitnessaddress: the P2SH-P2WPKH form of a wallet key
        sh = c.addwitnessaddress(c.getnewaddress())
        assert c.validateaddress(sh)["isvalid"]
        assert c.listwallets() == ["wallet.json"] and c.abortrescan() is False
    finally:
        node.stop()


def test_replacement_and_bumpfee(core, tmp_path):
    node = _node(core, tmp_path, "rbf", ["-mempoolreplacement=1", "-walletrbf=1"])
    plain = _node(core, tmp_path, "plain", [])
    try:
        c = client(node)
        fund(c, 110)
        _, _, ext = _key(core, b"rbf-dest")
        txid = c.sendtoaddress(ext, 3)
        before = c.gettransaction(txid)
        assert before["bip125-replaceable"] == "yes"
        bump = c.bumpfee(txid)
        assert bump["fee"] > bump["origfee"]
        pool = c.getrawmempool()
        assert bump["txid"] in pool and txid not in pool
        assert c.gettransaction(txid)["replaced_by_txid"] == bump["txid"]
        assert c.gettransaction(bump["txid"])["replaces_txid"] == txid
        with pytest.raises(RuntimeError, match="Insufficient totalFee"):
            c.bumpfee(bump["txid"], {"totalFee": 1})
        c.generatetoaddress(1, c.getnewaddress())
        assert c.gettransaction(bump["txid"])["confirmations"] == 1

        # without -walletrbf the wallet does not opt in, so there is nothing to bump
        p = client(plain)
        fund(p, 110)
        t2 = p.sendtoaddress(ext, 1)
        assert p.gettransaction(t2)["bip125-replaceable"] == "no"
        with pytest.raises(RuntimeError, match="not BIP 125 replaceable"):
            p.bumpfee(t2)
    finally:
        plain.stop()
        node.stop()


def test_replacement_rules_in_mempool(core, tmp_path):
    """BIP125 in AcceptToMemoryPool: opt-in, higher feerate, absolute fee, and the default off."""
    node = _node(core, tmp_path, "pool", ["-mempoolreplacement=1"])
    try:
        c = client(node)
        fund(c, 110)
        u = next(x for x in c.listunspent() if x["spendable"] and x["amount"] >= 10)
        _, _, ext = _key(core, b"pool-dest")

        def make(amount, seq):
            raw = c.createrawtransaction([{"txid": u["txid"], "vout": u["vout"], "sequence": seq}], {ext: amount})
            return c.signrawtransaction(raw)["hex"]

        first = make(u["amount"] - 0.1, 0xfffffffd)
        t1 = c.sendrawtransaction(first)
        with pytest.raises(RuntimeError, match="insufficient fee"):
            c.sendrawtransaction(make(u["amount"] - 0.05, 0xfffffffd))  # lower fee
        t3 = c.sendrawtransaction(make(u["amount"] - 0.2, 0xfffffffe))  # higher fee, final sequence
        pool = c.getrawmempool()
        assert t3 in pool and t1 not in pool
        with pytest.raises(RuntimeError, match="txn-mempool-conflict"):  # t3 did not opt in
            c.sendrawtransaction(make(u["amount"] - 0.5, 0xfffffffd))
        node.state.enable_replacement = False
        assert not node.state.enable_replacement
    finally:
        node.stop()


def test_accounts_and_sendfromaddress(core, tmp_path):
    node = _node(core, tmp_path, "acct", [])
    try:
        c = client(node)
        fund(c, 110)
        _, _, ext = _key(core, b"acct-dest")
        savings = c.getnewaddress("savings")
        c.sendtoaddress(savings, 20)
        c.generatetoaddress(1, c.getnewaddress())
        assert c.getreceivedbyaccount("savings") == 20
        assert c.getbalance("savings") == 20
        c.move("savings", "travel", 4, 1, "trip")
        assert c.getbalance("savings") == 16 and c.getbalance("travel") == 4
        assert any(e["category"] == "move" and e["otheraccount"] == "travel" for e in c.listtransactions("savings"))
        with pytest.raises(RuntimeError, match="Account has insufficient funds"):
            c.sendfrom("travel", ext, 5)
        t = c.sendfrom("savings", ext, 6, 1, "gift", "bob")
        g = c.gettransaction(t)
        assert g["details"][0]["account"] == "savings"
        assert c.getbalance("savings") == pytest.approx(16 - 6 - (-g["fee"]), abs=1e-8)
        accts = {r["account"]: r for r in c.listreceivedbyaccount(1, True)}
        assert accts["savings"]["amount"] == 20
        # sendfromaddress: only that address's coins, change back to it
        src = c.getnewaddress()
        c.sendtoaddress(src, 10)
        c.generatetoaddress(1, c.getnewaddress())
        with pytest.raises(RuntimeError, match="doesn't contain enough funds"):
            c.sendfromaddress(src, ext, 11)
        t = c.sendfromaddress(src, ext, 3)
        raw = c.getrawtransaction(t, 1)
        spent = {(v["txid"], v["vout"]) for v in raw["vin"]}
        assert len(spent) == 1
        outs = {o["scriptPubKey"]["addresses"][0]: o["value"] for o in raw["vout"]}
        assert outs[ext] == 3 and 6.9 < outs[src] < 7
    finally:
        node.stop()


def test_masterkeyinfo_and_pruned_funds(core, tmp_path):
    from nodexa_chain_core_amd.wallet.wallet import _bip32_master, ext_key_b58
    from nodexa_chain_core_amd.wallet import bip39

    words = BIP39_VECTORS[0][1]
    node = _node(core, tmp_path, "mk", [f"-mnemonic={words}", "-mnemonicpassphrase=TREZOR"])
    try:
        c = client(node)
        info = c.getmasterkeyinfo()
        k, cc = _bip32_master(bip39.to_seed(words, "TREZOR"))
        assert info["bip32_root_private"] == ext_key_b58(k, cc, "regtest")
        assert info["bip32_root_private"].startswith("tprv") and info["bip32_root_public"].startswith("tpub")
        assert info["account_derivation_path"] == "m/44'/1'/0'"
        assert info["account_extended_public_key"].startswith("tpub")

        fund(c, 110)
        secret, _, addr = _key(core, b"pruned")
        txid = c.sendtoaddress(addr, 2)
        c.generatetoaddress(1, c.getnewaddress())
        raw = c.getrawtransaction(txid)
        proof = c.gettxoutproof([txid])
        wif = core.base58check_encode(bytes([114]) + secret + b"\x01")
        c.removeprunedfunds(txid)  # it was ours as a send: drop it, then import it back by proof
        with pytest.raises(RuntimeError, match="Invalid or non-wallet"):
            c.gettransaction(txid)
        c.importprivkey(wif, "", False)
        c.importprunedfunds(raw, proof)
        assert c.gettransaction(txid)["confirmations"] == 1
        with pytest.raises(RuntimeError, match="does not exist"):
            c.removeprunedfunds("00" * 32)
        assert c.resendwallettransactions() == []
    finally:
        node.stop()


def test_standard_output_policy(core):
    from nodexa_chain_core_amd.chain import policy

    h = bytes(range(20))

    def tx_with(*outs):
        t = core.Transaction()
        t.vout = [core.TxOut(v, s) for v, s in outs]
        return t

    p2pkh = b"\x76\xa9\x14" + h + b"\x88\xac"
    assert policy.standard_outputs_reason(tx_with((1000, p2pkh))) == ""
    assert policy.standard_outputs_reason(tx_with((545, p2pkh))) == "dust"  # 182 bytes at 3000 sat/kB = 546
    assert policy.dust_threshold(p2pkh) == 546 and policy.dust_threshold(b"\x00\x14" + h) == 294
    assert policy.standard_outputs_reason(tx_with((0, b"\x6a\x04abcd"), (0, b"\x6a\x01x"))) == "multi-op-return"
    assert policy.standard_outputs_reason(tx_with((0, b"\x6a\x4c\x51" + b"x" * 81))) == "scriptpubkey"
    assert policy.standard_outputs_reason(tx_with((1000, b"\x51\xae"))) == "scriptpubkey"  # not a template
    ms = bytes([0x52]) + b"".join(b"\x21" + bytes([2]) + bytes(32) for _ in range(4)) + bytes([0x54, 0xae])
    assert policy.standard_outputs_reason(tx_with((1000, ms))) == "scriptpubkey"  # 2-of-4 bare multisig
    asset = core.asset_script_transfer(h, "ROSE", 5)
    assert policy.output_type(asset) == "asset" and policy.standard_outputs_reason(tx_with((0, asset))) == ""
    tag = core.asset_script_null_tag(h, "#KYC", 1)
    assert policy.output_type(tag) == "null_asset"
