"""Wallet, UTXO set, block connection / undo and AcceptToMemoryPool through a regtest node's
RPCs (the reference's functional wallet_basic / mempool_* / feature_reindex / rpc_blockchain
gettxoutsetinfo tests, for the subset this engine offers)."""
import os
import shutil

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import fund, mature_coin, spend



def _external(core):
    return core.base58check_encode(bytes([42]) + bytes(range(1, 21)))  # regtest PUBKEY_ADDRESS prefix


def test_balance_send_confirm_gettxout(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    ext = _external(core)
    fund(c)
    info = c.getwalletinfo()
    assert info["balance"] > 0 and info["immature_balance"] > 0
    bal = c.getbalance()
    assert bal == pytest.approx(mature_coin(c)["amount"])
    txid = c.sendtoaddress(ext, 10)
    assert txid in c.getrawmempool()
    entry = c.getmempoolentry(txid)
    fee = entry["fee"] if "fee" in entry else None
    # the change is unconfirmed, the spent coinbase is gone from the confirmed balance
    assert c.getbalance() == pytest.approx(0.0)
    assert c.getunconfirmedbalance() == pytest.approx(bal - 10 - (fee or 0), abs=0.01)
    before = c.gettxoutsetinfo()
    c.generatetoaddress(1, c.getnewaddress())
    assert c.getrawmempool() == []
    out = c.gettxout(txid, 0)
    assert out["value"] == 10 and out["confirmations"] == 1 and not out["coinbase"]
    assert out["scriptPubKey"]["addresses"] == [ext]
    after = c.gettxoutsetinfo()
    # +2 outputs of the spend, +coinbase outputs, -1 spent coinbase output
    assert after["height"] == before["height"] + 1
    assert after["bestblock"] != before["bestblock"] and after["hash_serialized_2"] != before["hash_serialized_2"]
    # spent outputs are gone; mempool-spent outputs are hidden unless include_mempool=false
    u = mature_coin(c)
    t2 = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], ext, 1.0))
    assert c.gettxout(u["txid"], u["vout"]) is None
    assert c.gettxout(u["txid"], u["vout"], False) is not None
    assert c.gettxout(t2, 0)["confirmations"] == 0


def test_consensus_rejections(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    ext = _external(core)
    w = c.getnewaddress()
    c.generatetoaddress(99, w)
    cb = [u for u in c.listunspent(1, 9999999, [w])]
    assert cb and not any(u["spendable"] for u in cb)
    first = min(cb, key=lambda u: -u["confirmations"])
    with pytest.raises(RuntimeError, match="premature-spend-of-coinbase"):
        c.sendrawtransaction(spend(c, first["txid"], first["vout"], first["amount"], ext, 1.0))
    c.generatetoaddress(1, w)
    good = spend(c, first["txid"], first["vout"], first["amount"], ext, 1.0)
    # a bad signature: flip a byte inside the DER signature of input 0
    tx = core.Transaction.deserialize(bytes.fromhex(good))
    vin = list(tx.vin)
    sig = bytearray(vin[0].script_sig)
    sig[10] ^= 1
    vin[0].script_sig = bytes(sig)
    tx.vin = vin
    with pytest.raises(RuntimeError, match="script-verify|SCRIPT_ERR|mandatory"):
        c.sendrawtransaction(tx.serialize(True).hex())
    # no fee at all: below the min relay fee
    nofee = spend(c, first["txid"], first["vout"], first["amount"], ext, first["amount"], fee=0)
    with pytest.raises(RuntimeError, match="min relay fee"):
        c.sendrawtransaction(nofee)
    # a fee above -maxtxfee (nAbsurdFee; the reference default is 1000 CLORE, lowered here to
    # 100 so a regtest coinbase can exceed it) is refused unless allowhighfees
    node.state.max_tx_fee = 100 * 100_000_000
    high = spend(c, first["txid"], first["vout"], first["amount"], ext, 1.0, fee=first["amount"] - 1.0)
    with pytest.raises(RuntimeError, match="absurdly-high-fee"):
        c.sendrawtransaction(high)
    txid = c.sendrawtransaction(good)
    # double spend of the same coin
    with pytest.raises(RuntimeError, match="txn-mempool-conflict"):
        c.sendrawtransaction(spend(c, first["txid"], first["vout"], first["amount"], ext, 2.0))
    c.generatetoaddress(1, w)
    raw = c.createrawtransaction([{"txid": first["txid"], "vout": first["vout"]}], {ext: 2.0})
    res = c.signrawtransaction(raw)
    assert not res["complete"] and "already spent" in res["errors"][0]["error"]
    with pytest.raises(RuntimeError, match="already in block chain"):
        c.sendrawtransaction(good)  # RPC_VERIFY_ALREADY_IN_CHAIN
    assert c.getrawtransaction(txid, True)["confirmations"] == 1


def test_block_with_invalid_spend_is_rejected(core, node_factory):  # noqa: F811
    """A block carrying a transaction with a bad signature fails ConnectBlock; the chain and the
    UTXO set stay where they were."""
    node, _ = node_factory()
    c = client(node)
    ext = _external(core)
    fund(c)
    u = mature_coin(c)
    tx = core.Transaction.deserialize(bytes.fromhex(spend(c, u["txid"], u["vout"], u["amount"], ext, 1.0)))
    vin = list(tx.vin)
    sig = bytearray(vin[0].script_sig)
    sig[10] ^= 1
    vin[0].script_sig = bytes(sig)
    tx.vin = vin
    node.state.add_to_mempool(tx, 1_000_000)  # bypass ATMP to get it into a template
    stats = c.gettxoutsetinfo()
    with pytest.raises(RuntimeError, match="mandatory-script-verify-flag-failed"):
        node.miner.generate(node.mining_script, 1)
    assert c.getblockcount() == 101
    assert c.gettxoutsetinfo()["hash_serialized_2"] == stats["hash_serialized_2"]


def test_reorg_restores_utxo_and_mempool(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    ext = _external(core)
    fund(c)
    txid = c.sendtoaddress(ext, 3)
    stats0 = c.gettxoutsetinfo()
    h = c.generatetoaddress(1, c.getnewaddress())[0]
    stats1 = c.gettxoutsetinfo()
    assert c.getrawmempool() == []
    c.invalidateblock(h)
    assert c.getblockcount() == 101
    assert c.gettxoutsetinfo()["hash_serialized_2"] == stats0["hash_serialized_2"]
    assert c.getrawmempool() == [txid]  # back in the pool (UpdateMempoolForReorg)
    c.reconsiderblock(h)
    assert c.getbestblockhash() == h
    assert c.gettxoutsetinfo()["hash_serialized_2"] == stats1["hash_serialized_2"]
    assert c.getrawmempool() == []
    # disconnect everything down to genesis: the UTXO set is empty again
    c.invalidateblock(c.getblockhash(1))
    s = c.gettxoutsetinfo()
    assert s["height"] == 0 and s["txouts"] == 0 and s["total_amount"] == 0
    c.reconsiderblock(c.getblockhash(1) if c.getblockcount() else h)
    assert c.gettxoutsetinfo()["hash_serialized_2"] == stats1["hash_serialized_2"]


def test_restart_reloads_and_rebuilds_utxo(core, node_factory, tmp_path):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    ext = _external(core)
    fund(c)
    c.sendtoaddress(ext, 2)
    c.generatetoaddress(1, c.getnewaddress())
    stats = c.gettxoutsetinfo()
    bal = c.getbalance()
    node.stop()
    chainstate = os.path.join(str(tmp_path), "regtest", "chainstate")
    assert os.path.exists(os.path.join(chainstate, "CURRENT"))  # the LevelDB-format UTXO store
    rev = os.path.join(str(tmp_path), "regtest", "blocks", "rev00000.dat")
    assert open(rev, "rb").read(4) == b"DROW"
    node, _ = node_factory()
    c = client(node)
    assert c.gettxoutsetinfo()["hash_serialized_2"] == stats["hash_serialized_2"]
    assert c.getbalance() == pytest.approx(bal)  # the wallet's keys were persisted
    node.stop()
    shutil.rmtree(chainstate)  # lost UTXO store: rebuilt by reconnecting the stored blocks
    node, _ = node_factory()
    c = client(node)
    assert c.gettxoutsetinfo()["hash_serialized_2"] == stats["hash_serialized_2"]


def test_segwit_outputs_sign_and_spend(core, node_factory):  # noqa: F811
    """P2WPKH and P2SH-P2WPKH outputs of wallet keys: found, signed (BIP143) and spent."""
    node, _ = node_factory()
    c = client(node)
    fund(c)
    addr = c.getnewaddress()
    h = core.base58check_decode(addr)[1:]
    p2wpkh = b"\x00\x14" + h
    p2sh = b"\xa9\x14" + core.hash160(p2wpkh) + b"\x87"
    wtx = node.wallet.send([(p2wpkh, 4 * 10**8), (p2sh, 3 * 10**8)])
    c.generatetoaddress(1, c.getnewaddress())
    mine = {(u["txid"], u["vout"]): u for u in c.listunspent()}
    wid = wtx[::-1].hex()
    assert (wid, 0) in mine and (wid, 1) in mine
    for n, amount in ((0, 4.0), (1, 3.0)):
        signed = spend(c, wid, n, amount, _external(core), 1.0)
        dec = c.decoderawtransaction(signed)
        assert dec["vin"][0].get("txinwitness"), dec  # witness carries sig + pubkey
        c.sendrawtransaction(signed)
    c.generatetoaddress(1, c.getnewaddress())
    assert c.getrawmempool() == []


def test_privkey_import_export(core, node_factory):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    addr = c.getnewaddress()
    wif = c.dumpprivkey(addr)
    assert core.base58check_decode(wif)[0] == 114 and len(core.base58check_decode(wif)) == 34
    c.importprivkey(wif)
    assert c.dumpprivkey(addr) == wif
    with pytest.raises(RuntimeError, match="Invalid private key"):
        c.importprivkey("notakey")
    with pytest.raises(RuntimeError):
        c.dumpprivkey(_external(core))
    # sendtoaddress with no funds
    with pytest.raises(RuntimeError, match="Insufficient funds"):
        c.sendtoaddress(addr, 1)


def test_history_rpcs_and_coin_control(core, node_factory, tmp_path):  # noqa: F811
    node, _ = node_factory()
    c = client(node)
    ext = _external(core)
    w = fund(c)
    txs = c.listtransactions("*", 1000)
    assert len(txs) == 101 and all(t["category"] in ("generate", "immature") for t in txs)
    assert sum(t["category"] == "generate" for t in txs) == 1
    txid = c.sendtoaddress(ext, 7, "rent")
    last = c.listtransactions("*", 1)[0]
    assert (last["txid"], last["category"], last["amount"], last["confirmations"]) == (txid, "send", -7, 0)
    assert last["fee"] < 0 and last["comment"] == "rent"
    c.generatetoaddress(1, w)
    t = c.gettransaction(txid)
    assert t["confirmations"] == 1 and t["amount"] == -7 and t["fee"] < 0 and t["details"][0]["address"] == ext
    # receive into a labelled address, then the received-by views
    mine = c.getnewaddress("savings")
    u = mature_coin(c)
    c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], mine, 3))
    h = c.generatetoaddress(1, w)[0]
    assert c.getreceivedbyaddress(mine) == 3
    assert any(r["address"] == mine and r["amount"] == 3 and r["account"] == "savings"
               for r in c.listreceivedbyaddress())
    assert mine in c.getaddressesbyaccount("savings") and c.getaccount(mine) == "savings"
    since = c.listsinceblock(c.getblockhash(c.getblockcount() - 1))
    assert any(e["address"] == mine for e in since["transactions"]) and since["lastblock"] == h
    # lockunspent keeps a coin out of coin selection
    coin = mature_coin(c)
    assert c.lockunspent(False, [{"txid": coin["txid"], "vout": coin["vout"]}])
    assert c.listlockunspent() == [{"txid": coin["txid"], "vout": coin["vout"]}]
    assert all((x["txid"], x["vout"]) != (coin["txid"], coin["vout"]) for x in c.listunspent())
    c.lockunspent(True)
    assert c.listlockunspent() == []
    # fundrawtransaction: wallet inputs + change for a bare output list, then sign and send
    raw = c.createrawtransaction([], {ext: 2.5})
    funded = c.fundrawtransaction(raw)
    assert funded["fee"] > 0 and funded["changepos"] >= 0
    sent = c.sendrawtransaction(c.signrawtransaction(funded["hex"])["hex"])
    assert sent in c.getrawmempool()
    # dumpwallet / importwallet round trip into a second wallet
    dump = str(tmp_path / "dump.txt")
    c.dumpwallet(dump)
    assert open(dump).read().count("# addr=") == len(node.wallet.keys)
    c.backupwallet(str(tmp_path / "backup.json"))
    assert (tmp_path / "backup.json").exists()
    c.settxfee(0.05)
    assert node.wallet.fee_rate == 5_000_000


def test_hd_keys_and_encryption(core, node_factory):  # noqa: F811
    from nodexa_chain_core_amd.wallet.wallet import _bip32_master, _ckd_priv

    # BIP32 test vector 1 (seed 000102...0f): master chain code and m/0' key
    k, c = _bip32_master(bytes(range(16)))
    assert c.hex() == "873dff81c02f525623fd1fe5167eac3a55a049de3d314bb42ee227ffed37d508"
    assert _ckd_priv(k, c, 0)[0].hex() == "edb2e14f9ee77d26dd93b4ecede8d16ed408ce149b6cd80b0715a2d911a0afea"
    node, _ = node_factory()
    c = client(node)
    info = c.getwalletinfo()
    assert "hdmasterkeyid" in info and "unlocked_until" not in info
    a1, a2 = c.getnewaddress(), c.getnewaddress()
    # -bip44 is the default: m/44'/coin_type'/account'/change/index, coin_type 1 off mainnet
    assert c.validateaddress(a1)["hdkeypath"] == "m/44'/1'/0'/0/0"
    assert c.validateaddress(a2)["hdkeypath"] == "m/44'/1'/0'/0/1"
    words = c.getmywords()["word_list"].split()
    assert len(words) == 12
    fund(c)
    wif = c.dumpprivkey(a1)
    # encrypt: locked afterwards; signing, dumping and fresh derivation need the passphrase
    c.encryptwallet("correct horse")
    info = c.getwalletinfo()
    assert info["unlocked_until"] == 0 and info["keypoolsize"] >= 100
    with pytest.raises(RuntimeError, match="-13"):
        c.dumpprivkey(a1)
    with pytest.raises(RuntimeError, match="-13"):
        c.sendtoaddress(_external(core), 1)
    assert c.validateaddress(c.getnewaddress())["ismine"]  # from the keypool while locked
    with pytest.raises(RuntimeError, match="-14"):
        c.walletpassphrase("wrong", 60)
    c.walletpassphrase("correct horse", 60)
    assert c.getwalletinfo()["unlocked_until"] > 0
    assert c.dumpprivkey(a1) == wif
    txid = c.sendtoaddress(_external(core), 1)
    assert txid in c.getrawmempool()
    c.generatetoaddress(1, a2)  # confirms the send (its change is ours)
    c.walletlock()
    with pytest.raises(RuntimeError, match="-13"):
        c.dumpprivkey(a1)
    c.walletpassphrasechange("correct horse", "battery staple")
    with pytest.raises(RuntimeError, match="-14"):
        c.walletpassphrase("correct horse", 10)
    # the encrypted wallet survives a restart
    node.stop()
    node, _ = node_factory()
    c = client(node)
    with pytest.raises(RuntimeError, match="-13"):
        c.dumpprivkey(a1)
    with pytest.raises(RuntimeError, match="-13"):
        c.getmywords()
    c.walletpassphrase("battery staple", 30)
    assert c.dumpprivkey(a1) == wif
    assert c.getwalletinfo()["balance"] > 0
    assert c.getmywords()["word_list"].split() == words  # the words were kept encrypted


# trezor/python-mnemonic vectors (passphrase "TREZOR"), as carried by the reference's
# src/test/data/bip39_vectors.json: entropy, mnemonic, seed, master xprv (used as data)
BIP39_VECTORS = [
    ["00000000000000000000000000000000",
     "abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon about",
     "c55257c360c07c72029aebc1b53c05ed0362ada38ead3e3e9efa3708e53495531f09a6987599d18264c1e1c92f2cf141630c7a3c4ab7c81b2f"
     "001698e7463b04",
     "xprv9s21ZrQH143K3h3fDYiay8mocZ3afhfULfb5GX8kCBdno77K4HiA15Tg23wpbeF1pLfs1c5SPmYHrEpTuuRhxMwvKDwqdKiGJS9XFKzUsAF"],
    ["ffffffffffffffffffffffffffffffff", "zoo zoo zoo zoo zoo zoo zoo zoo zoo zoo zoo wrong",
     "ac27495480225222079d7be181583751e86f571027b0497b5b5d11218e0a8a13332572917f0f8e5a589620c6f15b11c61dee327651a14c34"
     "e18231052e48c069",
     "xprv9s21ZrQH143K2V4oox4M8Zmhi2Fjx5XK4Lf7GKRvPSgydU3mjZuKGCTg7UPiBUD7ydVPvSLtg9hjp7MQTYsW67rZHAXeccqYqrsx8LcXnyd"],
    ["0000000000000000000000000000000000000000000000000000000000000000",
     "abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon abandon "
     "abandon abandon abandon abandon abandon abandon abandon abandon abandon art",
     "bda85446c68413707090a52022edd26a1c9462295029f2e60cd7c4f2bbd3097170af7a4d73245cafa9c3cca8d561a7c3de6f5d4a10be8ed2"
     "a5e608d68f92fcc8",
     "xprv9s21ZrQH143K32qBagUJAMU2LsHg3ka7jqMcV98Y7gVeVyNStwYS3U7yVVoDZ4btbRNf4h6ibWpY22iRmXq35qgLs79f312g2kj5539ebPM"],
    ["9f6a2878b2520799a44ef18bc7df394e7061a224d2c33cd015b157d746869863",
     "panda eyebrow bullet gorilla call smoke muffin taste mesh discover soft ostrich alcohol speed nation flash devote "
     "level hobby quick inner drive ghost inside",
     "72be8e052fc4919d2adf28d5306b5474b0069df35b02303de8c1729c9538dbb6fc2d731d5f832193cd9fb6aeecbc469594a70e3dd50811b5"
     "067f3b88b28c3e8d",
     "xprv9s21ZrQH143K2WNnKmssvZYM96VAr47iHUQUTUyUXH3sAGNjhJANddnhw3i3y3pBbRAVk5M5qUGFr4rHbEWwXgX4qrvrceifCYQJbbFDems"],
    ["f585c11aec520db57dd353c69554b21a89b20fb0650966fa0a9d6f74fd989d8f",
     "void come effort suffer camp survey warrior heavy shoot primary clutch crush open amazing screen patrol group "
     "space point ten exist slush involve unfold",
     "01f5bced59dec48e362f2c45b5de68b9fd6c92c6634f44d6d40aab69056506f0e35524a518034ddc1192e1dacd32c1ed3eaa3c3b131c88ed"
     "8e7e54c49a5d0998",
     "xprv9s21ZrQH143K39rnQJknpH1WEPFJrzmAqqasiDcVrNuk926oizzJDDQkdiTvNPr2FYDYzWgiMiC63YmfPAa2oPyNB23r2g7d1yiK6WpqaQS"],
]


def test_bip39_reference_vectors():
    from nodexa_chain_core_amd.wallet import bip39
    from nodexa_chain_core_amd.wallet.wallet import _bip32_master, ext_key_b58

    for entropy, words, seed, xprv in BIP39_VECTORS:
        assert bip39.from_entropy(bytes.fromhex(entropy)) == words
        assert bip39.check(words) and bip39.to_entropy(words).hex() == entropy
        s = bip39.to_seed(words, "TREZOR")
        assert s.hex() == seed
        k, c = _bip32_master(s)
        assert ext_key_b58(k, c, "main") == xprv
    assert not bip39.check("abandon " * 11 + "abandon")  # checksum
    assert not bip39.check("abandon " * 11 + "notaword")
    assert len(bip39.generate().split()) == 12


def test_wallet_from_mnemonic_is_deterministic(core, tmp_path):
    from test_p2p import _node

    words = BIP39_VECTORS[0][1]
    nodes = [_node(core, tmp_path, n, [f"-mnemonic={words}", "-mnemonicpassphrase=TREZOR"]) for n in ("m1", "m2")]
    try:
        c1, c2 = client(nodes[0]), client(nodes[1])
        assert [c1.getnewaddress() for _ in range(3)] == [c2.getnewaddress() for _ in range(3)]
        assert c1.getmywords() == {"word_list": words, "passphrase": "TREZOR"}
        assert c1.validateaddress(c1.getrawchangeaddress())["hdkeypath"] == "m/44'/1'/0'/1/0"
        dump = tmp_path / "dump.txt"
        c1.dumpwallet(str(dump))
        assert f"# mnemonic: {words}" in dump.read_text()
    finally:
        for n in nodes:
            n.stop()
    legacy = _node(core, tmp_path, "legacy", ["-bip44=0"])
    try:
        c = client(legacy)
        assert c.validateaddress(c.getnewaddress())["hdkeypath"] == "m/0'/0'/0'"
        with pytest.raises(RuntimeError, match="doesn't have 12 words"):
            c.getmywords()
    finally:
        legacy.stop()
