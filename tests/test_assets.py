"""Asset layer: names, scripts and verifier strings against the reference's own
test vectors (src/test/assets/asset_tests.cpp, verifier_string_tests.cpp — the name / expression
strings and expected answers are used as data), then a regtest node issuing, transferring,
reissuing, tagging and freezing through the RPCs, with reorg and restart."""
import os

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures

VALID = ["MIN", "MAX_ASSET_IS_30_CHARACTERS_LNG", "A_BCDEFGHIJKLMNOPQRSTUVWXY.Z", "0_12345678.9", "RAVEN.COIN",
         "CLORE.COIN", "RAVEN_COIN", "CLORE_COIN", "RVNSPYDER", "SPYDERRVN", "BLACK_CLORE", "SERVNOT", "ABC/A",
         "ABC/A/1", "ABC/A_1/1.A", "ABC/AB/XYZ/STILL/MAX/30/123456", "ABC#AZaz09", "ABC#abc123ABC@$%&*()[]{}-_.?:",
         "ABC/THING#_STILL_31_MAX-------_", "ABC~1", "ABC~MAX_OF_12_CR", "TEST/TEST~CHANNEL", "ABC!", "ABC^VOTE",
         "ABC^VOTING", "ABC^VOTING_IS_30_CHARACTERS_LN", "ABC/SUB/SUB/SUB/SUB^VOTE", "ABC/SUB/SUB/SUB/SUB/SUB/30^VOT",
         "ABC/SUB/SUB/SUB/SUB/SUB/31^VOTE", "ABC/SUB/SUB^VOTE", "TEST/UYTH#UNIQUE", "TEST/UYTH/SUB#UNIQUE",
         "TEST/UYTH/SUB~CHANNEL", "#ABC", "#ABC_TEST", "#ABC.TEST", "#ABC_IS_31_CHARACTERS_LENGTH_31",
         "#ABC/#TESTING", "#ABC/#TESTING_THIS", "#ABC/#SUB_IS_31_CHARACTERS_LENG", "#ABC/#A", "$ABC", "$ABC_A",
         "$ABC_IS_30_CHARACTERS_LENGTH30"]
INVALID = ["MAX_ASSET_IS_31_CHARACTERS_LONG", "NO", "nolower", "NO SPACE", "(#&$(&*^%$))", "_ABC", "ABC_", ".ABC",
           "ABC.", "AB..C", "A__BC", "A._BC", "AB_.C", "RVN", "RAVEN", "RAVENCOIN", "CLORE", "ABC//MIN_1", "ABC/",
           "ABC/NOTRAIL/", "ABC/_X", "ABC/X_", "ABC/.X", "ABC/X.", "ABC/X__X", "ABC/X..X", "ABC/X_.X", "ABC/X._X",
           "ABC/nolower", "ABC/NO SPACE", "ABC/(*#^&$%)", "ABC/AB/XYZ/STILL/MAX/30/OVERALL/1234", "ABC#no!bangs",
           "MIN#", "ABC#NO#HASH", "ABC#NO SPACE", "ABC#RESERVED/", "ABC#RESERVED~", "ABC#RESERVED^",
           "ABC~MAX_OF_12_CHR", "MIN~", "ABC~NO~TILDE", "ABC~_ANN", "ABC~ANN_", "ABC~.ANN", "ABC~ANN.", "ABC~X__X",
           "ABC~X._X", "ABC~X_.X", "ABC~X..X", "ABC^", "ABC^VOTING_IS_31_CHARACTERS_LN!",
           "ABC/SUB/SUB/SUB/SUB/SUB/32X^VOTE", "TEST/UYTH/SUB#UNIQUE^VOTE", "TEST/UYTH/SUB#UNIQUE#UNIQUE",
           "TEST/UYTH/SUB~CHANNEL^VOTE", "TEST/UYTH/SUB~CHANNEL^UNIQUE", "TEST/UYTH/SUB~CHANNEL!",
           "TEST/UYTH/SUB^VOTE!", "#ABC_IS_32_CHARACTERS_LEN_GTH_32", "#ABC^", "#ABC_.A", "#A", "#ABC!", "#_ABC",
           "#.ABC", "#ABC_", "#ABC.", "#ABC/TEST_", "#ABC/TEST.", "#ABC/TEST", "#ABC/#SUB_IS_32_CHARACTERS_LEN32",
           "$ABC_IS_32_CHARACTERSA_LENGTH_32", "$ABC/$NO", "$ABC/NO", "$ABC/#NO", "$ABC^NO", "$ABC~#NO", "$ABC#NO"]


def test_asset_names_match_reference_vectors(core):
    bad = [n for n in VALID if core.asset_name_type(n)[0] == "INVALID"]
    assert not bad, bad
    bad = [n for n in INVALID if core.asset_name_type(n)[0] != "INVALID"]
    assert not bad, bad
    assert core.asset_name_type("ABC")[0] == "ROOT" and core.asset_name_type("ABC/A")[0] == "SUB"
    assert core.asset_name_type("ABC#X")[0] == "UNIQUE" and core.asset_name_type("ABC!")[0] == "OWNER"
    assert core.asset_name_type("#ABC/#A")[0] == "SUB_QUALIFIER" and core.asset_name_type("$ABC")[0] == "RESTRICTED"
    assert core.asset_parent_name("ABC/SUB#TAG") == "ABC/SUB" and core.asset_parent_name("#A1C/#B") == "#A1C"


def test_verifier_strings_match_reference_vectors(core):
    vals = {"#KY_C": True, "#CI.A": False}
    assert core.bool_expr("#KY_C & !#CI.A", vals)
    for bad in ("#KY_C|#MISS", "BAD -- EXPRESSION -- BUST"):
        with pytest.raises(RuntimeError):
            core.bool_expr(bad, vals)
    good = core.strip_verifier_string("((#KYC & !#ABC) | #DEF & #GHI & #RET) | (#TEST)")
    assert good == "((KYC&!ABC)|DEF&GHI&RET)|(TEST)"
    names = ["KYC", "ABC", "DEF", "GHI", "RET", "TEST"]
    assert core.bool_expr(good, {n: True for n in names})
    assert not core.bool_expr(good, {n: False for n in names})
    for bad in ["", "(KYC", "(KYC)(", "(KYC)(&", "(KYC)(|", "(KYC)(|)", "(KYC)(&)", "(KYC)()", "KYC)", "$KYC",
                "KYC/SUB", "KYC$UNIQUE", "KYC~MSGCHANNEL", "KYC._", "KYC.|", "KYC &", "&", "(!)",
                "KYC&" * 19 + "KYC&KYC81", "(KYC && TEST)", "(KYC || TEST)", "(KYC |& TEST)", "(KYC &| TEST)",
                "KYC & | TEST", "KYC () TEST", "KYC ( ) TEST", "(true)", "!@#$%^&*()", "()"]:
        ok, err, _ = core.check_verifier_string(bad)
        assert not ok, bad
    assert core.check_verifier_string("true")[0]
    assert core.check_verifier_string("KYC & !BAD.A")[0]


def test_asset_scripts_roundtrip(core):
    h = bytes(range(20))
    ipfs = core.decode_asset_data("QmacSRmrkVmvJfbCpmU6pK72furJ8E8fbKHindrLxmYMQo")
    assert len(ipfs) == 34 and core.encode_asset_data(ipfs) == "QmacSRmrkVmvJfbCpmU6pK72furJ8E8fbKHindrLxmYMQo"
    new = core.asset_script_new(h, "ROSE", 1000 * 10**8, 2, 1, ipfs)
    assert new[:3] == b"\x76\xa9\x14" and new[25] == 0xC0 and new[-1] == 0x75
    a = core.parse_asset_script(new)
    assert (a["type"], a["name"], a["amount"], a["units"], a["reissuable"], a["has_ipfs"]) == \
        ("new_asset", "ROSE", 1000 * 10**8, 2, 1, 1)
    assert a["ipfs"] == ipfs and a["hash160"] == h
    t = core.parse_asset_script(core.asset_script_transfer(h, "ROSE", 5, b"\x11" * 32, 1700000000))
    assert (t["type"], t["amount"], t["message"], t["expire"]) == ("transfer_asset", 5, b"\x11" * 32, 1700000000)
    assert core.parse_asset_script(core.asset_script_owner(h, "ROSE!"))["amount"] == 10**8
    r = core.parse_asset_script(core.asset_script_reissue(h, "ROSE", 7, -1, 0))
    assert (r["type"], r["units"], r["reissuable"], r["ipfs"]) == ("reissue_asset", -1, 0, b"")
    tag = core.parse_null_asset_script(core.asset_script_null_tag(h, "#KYC", 1))
    assert tag == {"type": "tag", "hash160": h, "name": "#KYC", "flag": 1}
    assert core.parse_null_asset_script(core.asset_script_null_global("$ROSE", 0))["name"] == "$ROSE"
    assert core.parse_null_asset_script(core.asset_script_null_verifier("KYC"))["verifier"] == "KYC"
    # IsUnspendable: null asset data and zero-amount asset outputs never enter the UTXO set
    assert core.script_unspendable(core.asset_script_null_global("$ROSE", 0))
    assert core.script_unspendable(core.asset_script_transfer(h, "ROSE", 0))
    assert not core.script_unspendable(new)


def _ext(core):
    return core.base58check_encode(bytes([42]) + bytes(range(1, 21)))


def test_asset_lifecycle_regtest(core, node_factory):  # noqa: F811
    node, _ = node_factory(("-assetindex",))
    c = client(node)
    node.asset_index = False  # without -assetindex the per-address views answer with the reference's notice
    assert c.listaddressesbyasset("ROSE").startswith("_This rpc call is not functional unless -assetindex")
    node.asset_index = True
    w = c.getnewaddress()
    c.generatetoaddress(120, w)
    with pytest.raises(RuntimeError, match="Assets aren't active"):
        c.issue("ROSE", 1000)
    c.generatetoaddress(432 - 120, w)  # BIP9 on regtest: assets + messaging/restricted active from 433
    to = c.getnewaddress()
    c.issue("ROSE", 1000, to, "", 2, True)
    c.generatetoaddress(1, w)
    d = c.getassetdata("ROSE")
    assert (d["name"], d["amount"], d["units"], d["reissuable"], d["has_ipfs"]) == ("ROSE", 1000, 2, 1, 0)
    assert c.listmyassets() == {"ROSE": 1000, "ROSE!": 1}
    assert c.listassets() == ["ROSE", "ROSE!"]
    with pytest.raises(RuntimeError, match="already been used"):
        c.issue("ROSE", 5)
    # transfer part of it away; the change stays in the wallet
    ext = _ext(core)
    c.transfer("ROSE", 250.5, ext)
    c.generatetoaddress(1, w)
    assert c.listassetbalancesbyaddress(ext) == {"ROSE": 250.5}
    assert sum(c.listaddressesbyasset("ROSE").values()) == 1000
    assert c.listmyassets("ROSE") == {"ROSE": 749.5}
    with pytest.raises(RuntimeError, match="Insufficient asset funds"):
        c.transfer("ROSE", 5000, ext)
    # reissue (owner token spent and returned), then sub-asset and unique tokens under the owner token
    c.reissue("ROSE", 500, to, "", True, 4)
    c.generatetoaddress(1, w)
    reissue_tip = c.getbestblockhash()
    d = c.getassetdata("ROSE")
    assert d["amount"] == 1500 and d["units"] == 4
    c.issue("ROSE/PETAL", 10)
    c.generatetoaddress(1, w)
    c.issueunique("ROSE", ["A1", "B2"])
    c.generatetoaddress(1, w)
    assert {"ROSE/PETAL", "ROSE/PETAL!", "ROSE#A1", "ROSE#B2"} <= set(c.listassets())
    assert c.getassetdata("ROSE#A1")["amount"] == 1
    # qualifier, tag, restricted asset behind a verifier, freezes
    c.issuequalifierasset("#KYC", 2)
    c.generatetoaddress(1, w)
    holder = c.getnewaddress()
    c.addtagtoaddress("#KYC", holder)
    c.generatetoaddress(1, w)
    assert c.listtagsforaddress(holder) == ["#KYC"] and c.checkaddresstag(holder, "#KYC")
    assert c.listaddressesfortag("#KYC") == [holder]
    with pytest.raises(RuntimeError, match="verifier"):
        c.issuerestrictedasset("$ROSE", 100, "KYC", c.getnewaddress())  # untagged destination
    c.issuerestrictedasset("$ROSE", 100, "KYC", holder)
    c.generatetoaddress(1, w)
    assert c.getverifierstring("$ROSE") == "KYC" and c.getassetdata("$ROSE")["verifier_string"] == "KYC"
    assert c.isvalidverifierstring("KYC & !KYC") == "Valid Verifier"
    with pytest.raises(RuntimeError):
        c.isvalidverifierstring("NOPE")  # qualifier never issued
    c.freezeaddress("$ROSE", holder)
    c.generatetoaddress(1, w)
    assert c.checkaddressrestriction(holder, "$ROSE") and c.listaddressrestrictions(holder) == ["$ROSE"]
    with pytest.raises(RuntimeError, match="frozen"):
        c.transfer("$ROSE", 1, holder)
    c.unfreezeaddress("$ROSE", holder)
    c.freezerestrictedasset("$ROSE")
    c.generatetoaddress(1, w)
    assert not c.checkaddressrestriction(holder, "$ROSE") and c.checkglobalrestriction("$ROSE")
    assert c.listglobalrestrictions() == ["$ROSE"]
    c.removetagfromaddress("#KYC", holder)
    c.generatetoaddress(1, w)
    assert not c.checkaddresstag(holder, "#KYC")
    # reorg back below the reissue: amounts, units and everything after it revert; then forward again
    snapshot = {n: c.getassetdata(n) for n in c.listassets()}
    c.invalidateblock(reissue_tip)
    d = c.getassetdata("ROSE")
    assert d["amount"] == 1000 and d["units"] == 2
    assert c.getassetdata("$ROSE") is None and c.listglobalrestrictions() == []
    c.reconsiderblock(reissue_tip)
    assert {n: c.getassetdata(n) for n in c.listassets()} == snapshot
    # restart: the asset state is reloaded with the UTXO snapshot
    node.stop()
    node, _ = node_factory()
    assert not node.state.rebuilt  # loaded from the stored asset records, not replayed
    c = client(node)
    assert {n: c.getassetdata(n) for n in c.listassets()} == snapshot
    assert c.checkglobalrestriction("$ROSE")
    # a reference datadir: the same state as CAssetsDB / CRestrictedDB records (assets/,
    # assets/restricted) and none of this engine's asset records in chainstate/ -> imported at
    # start-up (chain/state._import_reference_assets), no replay
    before = _asset_state_view(node.state)
    height = node.state.coins_tip().height
    dd = node.state.datadir
    node.stop()
    _write_reference_asset_dbs(core, dd, before)
    db = core.LevelDB(os.path.join(dd, "chainstate"))
    db.write([(k, None) for k, _ in db.items(b"\x01", b"\x02")] + [(b"\x02assets.best", None)])
    db.close()
    node, _ = node_factory()
    assert not node.state.rebuilt and node.state.assets_import_height == height
    assert _asset_state_view(node.state) == before
    c = client(node)
    assert {n: c.getassetdata(n) for n in c.listassets()} == snapshot
    node.stop()
    node, _ = node_factory()  # the imported state was written in this engine's records
    assert not node.state.rebuilt and _asset_state_view(node.state) == before
    # after the import the engine owns the asset state: damaged engine records make the node replay
    # from genesis, never re-import the (now stale) reference assets/ databases
    node.stop()
    db = core.LevelDB(os.path.join(dd, "chainstate"))
    db.write([(k, None) for k, _ in db.items(b"\x01", b"\x02")] + [(b"\x02assets.best", None)])
    db.close()
    node, _ = node_factory()
    assert node.state.rebuilt and node.state.assets_import_height == -1
    assert _asset_state_view(node.state) == before  # the replay rebuilds the same state
    node.stop()
    node, _ = node_factory()  # and is the engine's own from then on: loaded, no import height
    assert not node.state.rebuilt and node.state.assets_import_height == -1
    assert _asset_state_view(node.state) == before


def _asset_state_view(state):
    st = state.assets
    return {"metas": {n: st.get(n) for n in st.names()}, "balances": sorted(st.balances()),
            "tags": sorted(st.tags()), "restrictions": sorted(st.restrictions()),
            "global": sorted(st.global_restrictions()),
            "verifiers": {n: st.verifier(n) for n in st.names() if st.verifier(n) is not None}}


def _write_reference_asset_dbs(core, datadir, view):
    """The reference's record layout, serialized here from its sources (not through the importer):
    src/assets/assetdb.cpp:17-41 (CAssetsDB keys), assettypes.h:59-185 (CDatabasedAssetData /
    CNewAsset / ReadWriteAssetHash), restricteddb.cpp:10-100 (CRestrictedDB keys, int8 1 values)."""
    import struct

    def cs(n):
        return bytes([n]) if n < 253 else b"\xfd" + struct.pack("<H", n)

    def s(b):
        b = b.encode() if isinstance(b, str) else b
        return cs(len(b)) + b

    def addr(h):
        return core.base58check_encode(bytes([42]) + h)

    a, r = [], []
    for name, m in view["metas"].items():
        v = s(name) + struct.pack("<qbbb", m["amount"], m["units"], m["reissuable"], m["has_ipfs"])
        if m["has_ipfs"] == 1:
            ipfs = m["ipfs"]
            v += (b"\x12" + s(ipfs[2:])) if len(ipfs) == 34 else (b"\x54" + s(ipfs))
        a.append((b"A" + s(name), v + struct.pack("<i", m["height"]) + m["block"]))
    for name, h, q in view["balances"]:
        a.append((b"B" + s(name) + s(addr(h)), struct.pack("<q", q)))
        a.append((b"C" + s(addr(h)) + s(name), struct.pack("<q", q)))  # the reverse index (not needed)
    for name, ver in view["verifiers"].items():
        r.append((b"V" + s(name), s(ver)))
    for tag, h in view["tags"]:
        r.append((b"T" + s(addr(h)) + s(tag), b"\x01"))
        r.append((b"Q" + s(tag) + s(addr(h)), b"\x01"))
    for name, h in view["restrictions"]:
        r.append((b"R" + s(addr(h)) + s(name), b"\x01"))
    for name in view["global"]:
        r.append((b"G" + s(name), b"\x01"))
    for sub, recs in (("assets", a), (os.path.join("assets", "restricted"), r)):
        db = core.LevelDB(os.path.join(datadir, sub))
        db.write(recs)
        db.close()


def test_asset_consensus_rejections(core, node_factory):  # noqa: F811
    """Hand-built transactions that break the asset rules are refused by AcceptToMemoryPool."""
    node, _ = node_factory()
    c = client(node)
    w = c.getnewaddress()
    c.generatetoaddress(432, w)
    to = c.getnewaddress()
    c.issue("LILY", 100, to)
    c.generatetoaddress(1, w)
    aw = node.asset_wallet
    coin = aw.unspent("LILY")[0]
    h = coin["hash160"]
    TxOut = core.TxOut

    def attempt(outs):
        tx, _ = node.wallet.fund_and_sign(outs, [], [coin])
        return node.state.accept_to_mempool(tx, test_only=True)

    ok, why, _ = attempt([TxOut(0, core.asset_script_transfer(h, "LILY", 60 * 10**8))])
    assert not ok and "Assets would be burnt" in why
    ok, why, _ = attempt([TxOut(0, core.asset_script_transfer(h, "LILY", 150 * 10**8))])
    assert not ok and "Assets would be burnt" in why
    ok, why, _ = attempt([TxOut(0, core.asset_script_transfer(h, "LILY", 100 * 10**8)),
                          TxOut(0, core.asset_script_transfer(h, "OTHER", 10**8))])
    assert not ok and why == "bad-txns-transfer-asset-not-exist"
    ok, why, _ = attempt([TxOut(0, core.asset_script_transfer(h, "LILY", 100 * 10**8)),
                          TxOut(0, core.asset_script_transfer(h, "LILY!", 10**8))])
    assert not ok and "don't have" in why
    ok, why, _ = attempt([TxOut(5, core.asset_script_transfer(h, "LILY", 100 * 10**8))])
    assert not ok and why == "bad-txns-asset-transfer-amount-isn't-zero"
    ok, why, _ = attempt([TxOut(0, core.asset_script_transfer(h, "LILY", 100 * 10**8))])
    assert ok, why
    # a new-asset output without its owner token / burn is not an issuance
    ok, why, _ = attempt([TxOut(0, core.asset_script_transfer(h, "LILY", 100 * 10**8)),
                          TxOut(0, core.asset_script_new(h, "FREE", 10**8))])
    assert not ok and why == "bad-txns-bad-asset-transaction"
