"""Reference wallet.dat import (csrc/store/bdb.cpp, wallet/walletdb.py; the reference's wallet
records: src/wallet/walletdb.cpp:244-590).

The oracle for the page format is the system's own Berkeley DB library (libdb-5.3, driven through
ctypes only to WRITE fixture files here; btree version 9, the on-disk format of the BDB 4.8 the
reference links): files it writes must read back record-for-record through the native reader. The
wallet records are built with the reference's serializations (compact-size strings and vectors,
DER CPrivKey, CMasterKey, CHDChain, CKeyMetadata, CKeyPool); the reference ships no wallet.dat,
so a record layout the reference's own code would write but these fixtures do not cover is
parity unpinned.
"""
import ctypes
import ctypes.util
import os
import random
import struct

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures


def _libdb():
    for name in ("libdb-5.3.so", ctypes.util.find_library("db-5.3"), ctypes.util.find_library("db")):
        if not name:
            continue
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    return None


LIBDB = _libdb()
needs_libdb = pytest.mark.skipif(LIBDB is None, reason="libdb (Berkeley DB) not installed: no fixture writer")


class _DBT(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("size", ctypes.c_uint32), ("ulen", ctypes.c_uint32),
                ("dlen", ctypes.c_uint32), ("doff", ctypes.c_uint32), ("app_data", ctypes.c_void_p),
                ("flags", ctypes.c_uint32)]


def _dbt(b: bytes, keep: list):
    buf = ctypes.create_string_buffer(b, len(b))
    keep.append(buf)
    return _DBT(ctypes.cast(buf, ctypes.c_void_p), len(b), 0, 0, 0, None, 0)


def bdb_write(path: str, records, subdb: bytes = b"main", delete=(), lorder: int = 0, pagesize: int = 0) -> None:
    """A btree file written by libdb itself (DB->open(DB_BTREE, DB_CREATE), DB->put, DB->del);
    `lorder` 4321 writes a big-endian file, `pagesize` overrides the page size."""
    db = ctypes.c_void_p()
    assert LIBDB.db_create(ctypes.byref(db), None, 0) == 0
    if lorder:
        assert LIBDB.__db_set_lorder(db, lorder) == 0
    if pagesize:
        assert LIBDB.__db_set_pagesize(db, pagesize) == 0
    assert LIBDB.__db_open_pp(db, None, path.encode(), subdb, 1, 1, 0o600) == 0  # DB_BTREE, DB_CREATE
    keep: list = []
    for k, v in records:
        assert LIBDB.__db_put_pp(db, None, ctypes.byref(_dbt(k, keep)), ctypes.byref(_dbt(v, keep)), 0) == 0
    for k in delete:
        assert LIBDB.__db_del_pp(db, None, ctypes.byref(_dbt(k, keep)), 0) == 0
    assert LIBDB.__db_close_pp(db, 0) == 0


# ---------------------------------------------------------------- the reference's serializations
def cs(n: int) -> bytes:
    if n < 253:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + struct.pack("<H", n)
    return b"\xfe" + struct.pack("<I", n)


def vec(b: bytes) -> bytes:
    return cs(len(b)) + b


def rkey(t: str, *parts: bytes) -> bytes:
    return vec(t.encode()) + b"".join(parts)


def der_privkey(core, secret: bytes) -> bytes:
    """CPrivKey as ec_privkey_export_der writes a compressed key (src/key.cpp:69-95): the fixed
    prefix, the secret, the curve parameters, the public key."""
    begin = bytes([0x30, 0x81, 0xD3, 0x02, 0x01, 0x01, 0x04, 0x20])
    middle = bytes(141)  # the curve parameter block (not read back by any loader)
    return begin + secret + middle + b"\xa1\x24\x03\x22\x00" + core.secp_pubkey_create(secret, True)


def key_record(core, secret: bytes):
    pub = core.secp_pubkey_create(secret, True)
    der = der_privkey(core, secret)
    return rkey("key", vec(pub)), vec(der) + core.sha256d(pub + der)


def keymeta_record(pub: bytes, created: int, path: str, seed_id: bytes):
    return rkey("keymeta", vec(pub)), struct.pack("<iq", 10, created) + vec(path.encode()) + seed_id


def hdchain_record(ext: int, internal: int, seed_id: bytes, bip44: bool, version: int = 3):
    v = struct.pack("<iI", version, ext) + seed_id
    if version >= 2:
        v += struct.pack("<I", internal)
    if version == 3:
        v += bytes([bip44])
    return rkey("hdchain"), v


def pool_record(idx: int, pub: bytes, internal: bool = False):
    return rkey("pool", struct.pack("<q", idx)), struct.pack("<iq", 2010000, 1_600_000_000) + vec(pub) + bytes([internal])


# ---------------------------------------------------------------- the native page reader
@needs_libdb
def test_bdb_reader_matches_libdb(core, tmp_path):
    """Records of every shape libdb lays out (inline items, overflow chains, multi-level trees,
    deleted keys, two sub-databases in one file) read back exactly and in key order."""
    rng = random.Random(7)
    recs = {}
    for _ in range(2500):
        k = rng.randbytes(rng.randint(1, 40))
        recs[k] = rng.randbytes(rng.choice([0, 5, 50, 300, 2000, 9000]))
    gone = list(recs)[::7]
    p = str(tmp_path / "t.dat")
    bdb_write(p, list(recs.items()), delete=gone)
    other = {b"a": b"1", b"b" * 3000: b"2" * 5000}
    bdb_write(p, list(other.items()), subdb=b"other")
    for k in gone:
        del recs[k]
    assert sorted(core.bdb_databases(p)) == ["main", "other"]
    got = core.bdb_read(p, "main")
    assert [k for k, _ in got] == sorted(recs)
    assert dict(got) == recs
    assert dict(core.bdb_read(p, "other")) == other
    with pytest.raises(RuntimeError, match="no sub-database"):
        core.bdb_read(p, "nope")


@needs_libdb
@pytest.mark.parametrize("lorder,pagesize", [(4321, 0), (1234, 512), (4321, 65536)])
def test_bdb_reader_byte_orders_and_page_sizes(core, tmp_path, lorder, pagesize):
    """Big-endian files (a wallet.dat written on another host) and the smallest and largest page
    sizes read back exactly."""
    rng = random.Random(lorder + pagesize)
    recs = {rng.randbytes(rng.randint(1, 30)): rng.randbytes(rng.choice([1, 40, 700, 5000])) for _ in range(400)}
    p = str(tmp_path / "t.dat")
    bdb_write(p, list(recs.items()), lorder=lorder, pagesize=pagesize)
    assert dict(core.bdb_read(p, "main")) == recs


@needs_libdb
def test_bdb_reader_refuses_damage(core, tmp_path):
    p = str(tmp_path / "t.dat")
    bdb_write(p, [(bytes([i]) * 8, bytes(600)) for i in range(200)])
    raw = bytearray(open(p, "rb").read())
    junk = tmp_path / "junk.dat"
    junk.write_bytes(b"\0" * 8192)
    with pytest.raises(RuntimeError, match="magic"):
        core.bdb_read(str(junk), "main")
    cut = tmp_path / "cut.dat"
    cut.write_bytes(bytes(raw[:4096 * 2]))  # the tree's pages are gone
    with pytest.raises(RuntimeError):
        core.bdb_read(str(cut), "main")
    bad = bytearray(raw)
    ps = struct.unpack_from("<I", bad, 20)[0]
    for pg in range(1, len(bad) // ps):  # point every leaf item past its page
        if bad[pg * ps + 25] == 5:
            n = struct.unpack_from("<H", bad, pg * ps + 20)[0]
            for i in range(n):
                struct.pack_into("<H", bad, pg * ps + 26 + 2 * i, ps - 1)
    badp = tmp_path / "bad.dat"
    badp.write_bytes(bytes(bad))
    with pytest.raises(RuntimeError, match="past the page"):
        core.bdb_read(str(badp), "main")


# ---------------------------------------------------------------- wallet records -> JSON wallet
def _params():
    from nodexa_chain_core_amd.chain.state import make_params

    return make_params("regtest")


def _derive44(seed: bytes, chain: int, idx: int, coin: int = 1) -> bytes:
    from nodexa_chain_core_amd.wallet.wallet import _bip32_master, _ckd_priv

    k, c = _bip32_master(seed)
    for i, hard in ((44, True), (coin, True), (0, True), (chain, False), (idx, False)):
        k, c = _ckd_priv(k, c, i, hard)
    return k


def _bip44_wallet_records(core, mnemonic: str, passphrase: str, n_ext: int, crypt=None):
    """A reference BIP44 wallet: n_ext derived receive keys, one change key, keymeta, labels, a
    pool entry, an HD chain, BIP39 words / passphrase / seed; `crypt` = (master, word_hash) writes
    the encrypted forms (EncryptWallet: ckey + mkey + cbip39*)."""
    from nodexa_chain_core_amd.wallet import bip39

    seed = bip39.to_seed(mnemonic, passphrase)
    seed_id = core.hash160(core.secp_pubkey_create(_derive44(seed, 0, 0), True))  # any 20-byte id
    recs, secrets = [], []
    for chain, idx in [(0, i) for i in range(n_ext)] + [(1, 0)]:
        sec = _derive44(seed, chain, idx)
        pub = core.secp_pubkey_create(sec, True)
        secrets.append(sec)
        if crypt is None:
            recs.append(key_record(core, sec))
        else:
            master = crypt[0]
            recs.append((rkey("ckey", vec(pub)), vec(core.aes256_cbc_encrypt(master, core.sha256d(pub)[:16], sec))))
        recs.append(keymeta_record(pub, 1_600_000_000 + idx, f"m/44'/1'/0'/{chain}/{idx}", seed_id))
    recs.append(hdchain_record(n_ext, 1, seed_id, True))
    if crypt is None:
        recs.append((rkey("bip39words"), core.sha256d(mnemonic.encode()) + vec(mnemonic.encode())))
        recs.append((rkey("bip39passphrase"), vec(passphrase.encode())))
        recs.append((rkey("bip39vchseed"), vec(seed)))
    else:
        master, wh = crypt
        enc = lambda b: core.aes256_cbc_encrypt(master, wh[:16], b)  # noqa: E731
        recs.append((rkey("cbip39words"), wh + vec(enc(mnemonic.encode()))))
        recs.append((rkey("cbip39passphrase"), vec(enc(passphrase.encode()))))
        recs.append((rkey("cbip39vchseed"), vec(enc(seed))))
    return recs, secrets, seed


def _p2pkh_addr(core, params, sec: bytes) -> str:
    return core.base58check_encode(bytes([params.pubkey_prefix]) + core.hash160(core.secp_pubkey_create(sec, True)))


@needs_libdb
def test_import_plain_bip44_wallet(core, tmp_path):
    from nodexa_chain_core_amd.wallet import bip39
    from nodexa_chain_core_amd.wallet.wallet import Wallet

    params = _params()
    words = bip39.generate(128)
    recs, secrets, seed = _bip44_wallet_records(core, words, "pp", 3)
    a0 = _p2pkh_addr(core, params, secrets[0])
    recs.append((rkey("name", vec(a0.encode())), vec(b"savings")))
    recs.append((rkey("purpose", vec(a0.encode())), vec(b"receive")))
    recs.append(pool_record(1, core.secp_pubkey_create(secrets[2], True)))
    redeem = b"\x51\x21" + core.secp_pubkey_create(secrets[1], True) + b"\x51\xae"
    recs.append((rkey("cscript", core.hash160(redeem)), vec(redeem)))
    watch_spk = b"\x76\xa9\x14" + bytes(range(20)) + b"\x88\xac"
    recs.append((rkey("watchs", vec(watch_spk)), b"1"))
    recs.append((rkey("tx", bytes(32)), b"\x01\x02"))
    recs.append((rkey("version"), struct.pack("<i", 2010000)))
    dat = str(tmp_path / "wallet.dat")
    bdb_write(dat, recs)

    js = str(tmp_path / "wallet.json")
    w = Wallet(None, params, js, import_from=dat)
    rep = w.import_report
    assert rep["keys"] == 4 and rep["labels"] == 1 and rep["pool"] == 1 and rep["hd"]["bip44"], rep
    assert rep["not_imported"] == {"tx": 1}, rep
    assert w.dump_privkey(a0) == w.encode_wif(secrets[0])
    assert w.labels[core.hash160(core.secp_pubkey_create(secrets[0], True))] == "savings"
    assert w.mnemonic() == (words, "pp")
    assert core.hash160(redeem) in w.redeem_scripts and watch_spk in w.watch
    # the pool hands out the reference's reserved key first, then the chain continues at index 3
    assert w.new_address("x") == _p2pkh_addr(core, params, secrets[2])
    assert w.new_address("y") == _p2pkh_addr(core, params, _derive44(seed, 0, 3))
    # the JSON wallet now stands on its own: reopened without the .dat
    os.remove(dat)
    w2 = Wallet(None, params, js)
    assert w2.dump_privkey(a0) == w.encode_wif(secrets[0]) and w2.mnemonic() == (words, "pp")


@needs_libdb
def test_import_encrypted_bip44_wallet(core, tmp_path):
    """An encrypted reference wallet imports locked; the reference passphrase unlocks it (the
    master key derivation and AES-256-CBC are CCrypter's) and yields the keys, the BIP39 words
    and the seed the HD chain continues from."""
    from nodexa_chain_core_amd.wallet import bip39
    from nodexa_chain_core_amd.wallet.wallet import Wallet, WalletError

    params = _params()
    master, salt, rounds = os.urandom(32), os.urandom(8), 1000
    words = bip39.generate(128)
    wh = core.sha256d(b"word hash")
    recs, secrets, seed = _bip44_wallet_records(core, words, "", 2, crypt=(master, wh))
    k, iv = core.bytes_to_key_sha512("correct horse", salt, rounds)
    recs.append((rkey("mkey", struct.pack("<I", 1)),
                 vec(core.aes256_cbc_encrypt(k, iv, master)) + vec(salt) + struct.pack("<II", 0, rounds) + vec(b"")))
    dat = str(tmp_path / "wallet.dat")
    bdb_write(dat, recs)
    js = str(tmp_path / "wallet.json")
    w = Wallet(None, params, js, import_from=dat)
    assert w.import_report["crypted_keys"] == 3 and w.import_report["encrypted"]
    assert w.locked
    a0 = _p2pkh_addr(core, params, secrets[0])
    with pytest.raises(WalletError):
        w.dump_privkey(a0)
    with pytest.raises(WalletError, match="incorrect"):
        w.unlock("wrong")
    w.unlock("correct horse")
    assert w.dump_privkey(a0) == w.encode_wif(secrets[0])
    assert w.mnemonic() == (words, "")
    assert w.new_address() == _p2pkh_addr(core, params, _derive44(seed, 0, 2))
    w.lock_wallet()
    w2 = Wallet(None, params, js)  # reopened from JSON: still the reference's passphrase and IVs
    assert w2.locked
    w2.unlock("correct horse")
    assert w2.mnemonic() == (words, "") and w2.dump_privkey(a0) == w.encode_wif(secrets[0])


@needs_libdb
def test_import_legacy_hd_wallet(core, tmp_path):
    """A -bip44=0 reference wallet (the 0.15 layout): the seed is a wallet key named by the HD
    chain's seed id; keys continue at m/0'/0'/<external counter>'."""
    from nodexa_chain_core_amd.wallet.wallet import Wallet, _bip32_master, _ckd_priv

    params = _params()
    seed = os.urandom(32)
    while not core.secp_seckey_valid(seed):
        seed = os.urandom(32)
    seed_id = core.hash160(core.secp_pubkey_create(seed, True))

    def legacy(i):
        k, c = _bip32_master(seed)
        for j in (0, 0, i):
            k, c = _ckd_priv(k, c, j)
        return k

    recs = [key_record(core, seed), key_record(core, legacy(0)), key_record(core, legacy(1)),
            hdchain_record(2, 0, seed_id, False, version=2)]
    dat = str(tmp_path / "wallet.dat")
    bdb_write(dat, recs)
    w = Wallet(None, params, str(tmp_path / "w.json"), import_from=dat)
    assert w.import_report["hd"] == {"bip44": False, "external": 2, "internal": 0}
    assert w.new_address() == _p2pkh_addr(core, params, legacy(2))


@needs_libdb
def test_import_uncompressed_keys_refused_or_kept_aside(core, tmp_path):
    """A wallet.dat with an uncompressed key: refused by default (its funds would drop out of the
    wallet); with keep_uncompressed (-walletkeepuncompressed=1) the rest is imported and the
    uncompressed key is saved verbatim beside it, surviving a reload."""
    from nodexa_chain_core_amd.wallet.wallet import Wallet, WalletError

    params = _params()
    comp, unc = bytes([3]) * 32, bytes([4]) * 32
    upub = core.secp_pubkey_create(unc, False)
    uder = bytes([0x30, 0x82, 0x01, 0x13, 0x02, 0x01, 0x01, 0x04, 0x20]) + unc + bytes(141) + b"\xa1\x44\x03\x42\x00" + upub
    recs = [key_record(core, comp), (rkey("key", vec(upub)), vec(uder) + core.sha256d(upub + uder))]
    dat = str(tmp_path / "wallet.dat")
    bdb_write(dat, recs)
    js = str(tmp_path / "w.json")
    with pytest.raises(WalletError, match="uncompressed"):
        Wallet(None, params, js, import_from=dat)
    assert not os.path.exists(js)
    w = Wallet(None, params, js, import_from=dat, keep_uncompressed=True)
    assert w.import_report["keys"] == 1 and w.import_report["uncompressed_skipped"] == 1
    assert w.uncompressed == {upub: {"sec": unc}}
    w2 = Wallet(None, params, js)
    assert w2.uncompressed == {upub: {"sec": unc}} and len(w2.keys) == 1


@needs_libdb
def test_import_rejects_corrupt_key_record(core, tmp_path):
    from nodexa_chain_core_amd.wallet.wallet import Wallet

    k, v = key_record(core, bytes([1]) * 32)
    v = v[:-1] + bytes([v[-1] ^ 1])  # the sha256d(pub || privkey) checksum no longer matches
    dat = str(tmp_path / "wallet.dat")
    bdb_write(dat, [(k, v)])
    with pytest.raises(ValueError, match="corrupt"):
        Wallet(None, _params(), str(tmp_path / "w.json"), import_from=dat)
    assert not os.path.exists(tmp_path / "w.json")


@needs_libdb
def test_node_imports_reference_wallet_dat(core, node_factory, tmp_path):  # noqa: F811
    """A datadir holding the reference's wallet.dat and no JSON wallet: the node imports it at
    start-up (once) and serves its keys over the wallet RPCs."""
    from nodexa_chain_core_amd.wallet import bip39

    params = _params()
    words = bip39.generate(128)
    recs, secrets, _ = _bip44_wallet_records(core, words, "", 2)
    d = tmp_path / "regtest"
    d.mkdir(exist_ok=True)
    bdb_write(str(d / "wallet.dat"), recs)
    node, _ = node_factory()
    c = client(node)
    a0 = _p2pkh_addr(core, params, secrets[0])
    assert c.validateaddress(a0)["ismine"] is True
    assert c.dumpprivkey(a0) == core.base58check_encode(bytes([114]) + secrets[0] + b"\x01")  # regtest WIF
    assert os.path.exists(d / "wallet.json") and os.path.exists(d / "wallet.dat")


# ------------------------------------------------------------------ export (wallet/walletdb.py)
def _libdb_records(path: str):
    """Every (key, value) of sub-database "main" read by libdb itself (DB->open + a DB_NEXT cursor),
    after DB->verify of the whole file."""
    db = ctypes.c_void_p()
    assert LIBDB.db_create(ctypes.byref(db), None, 0) == 0
    assert LIBDB.__db_verify_pp(db, path.encode(), None, None, 0) == 0  # DB->verify closes the handle
    db = ctypes.c_void_p()
    assert LIBDB.db_create(ctypes.byref(db), None, 0) == 0
    assert LIBDB.__db_open_pp(db, None, path.encode(), b"main", 1, 0, 0) == 0  # DB_BTREE
    dbc = ctypes.c_void_p()
    assert LIBDB.__db_cursor_pp(db, None, ctypes.byref(dbc), 0) == 0
    out = []
    while True:
        k, v = _DBT(), _DBT()
        if LIBDB.__dbc_get_pp(dbc, ctypes.byref(k), ctypes.byref(v), 16) != 0:  # DB_NEXT
            break
        out.append((ctypes.string_at(k.data, k.size), ctypes.string_at(v.data, v.size)))
    LIBDB.__db_close_pp(db, 0)
    return out


def test_bdb_writer_pages_and_overflow(core, tmp_path):
    """The native writer (csrc/store/bdb.cpp) over records that need several leaf pages, an
    internal level and overflow chains; read back by this reader (and by libdb when present)."""
    import random

    rng = random.Random(3)
    recs = {rng.randbytes(rng.randint(1, 60)): rng.randbytes(rng.choice([1, 40, 300, 1500, 9000])) for _ in range(700)}
    path = str(tmp_path / "w.dat")
    core.bdb_write(path, list(recs.items()))
    assert core.bdb_read(path, "main") == sorted(recs.items())
    assert core.bdb_databases(path) == ["main"]
    if LIBDB is not None:
        assert _libdb_records(path) == sorted(recs.items())
    with pytest.raises(Exception):
        core.bdb_write(path, [(b"a", b"1"), (b"a", b"2")])  # duplicate key


@needs_libdb
def test_bdb_writer_file_takes_libdb_updates(core, tmp_path):
    """libdb inserts into a file this writer made (page splits included), and both readers agree."""
    path = str(tmp_path / "w.dat")
    base = [(b"k%04d" % i, b"v" * 30) for i in range(200)]
    core.bdb_write(path, base)
    more = [(b"m%04d" % i, bytes([i % 256]) * 90) for i in range(300)]
    bdb_write(path, more)
    assert core.bdb_read(path, "main") == sorted(base + more) == _libdb_records(path)


def _export_reimport(core, params, w, tmp_path, name="out.dat"):
    from nodexa_chain_core_amd.wallet.walletdb import write_wallet_dat
    from nodexa_chain_core_amd.wallet.wallet import Wallet

    dat = str(tmp_path / name)
    n = write_wallet_dat(w, dat)
    assert n > 0
    if LIBDB is not None:
        assert len(_libdb_records(dat)) == n
    return Wallet(None, params, str(tmp_path / (name + ".json")), import_from=dat), dat


def test_export_plain_bip44_wallet_round_trips(core, tmp_path):
    """A wallet made here (BIP44 / BIP39) written as a reference wallet.dat and imported again:
    the same keys, labels, words, keypool and the HD chain continuing at the same index."""
    from nodexa_chain_core_amd.wallet.wallet import Wallet
    from nodexa_chain_core_amd.wallet.walletdb import read_wallet_dat

    params = _params()
    w = Wallet(None, params, str(tmp_path / "w.json"))
    a1 = w.new_address("alice")
    a2 = w.new_address("")
    w.keypool_refill(3)
    w2, dat = _export_reimport(core, params, w, tmp_path)
    ref = read_wallet_dat(dat)
    assert ref["version"] == 4040402 and ref["hdchain"]["version"] == 3 and ref["hdchain"]["bip44"]
    assert ref["hdchain"]["seed_id"] == core.hash160(b"")  # what the reference writes for a BIP39 seed
    assert len(ref["keys"]) == len(w.keys) and len(ref["pool"]) == len(w.pool) == 3
    assert ref["names"][a1] == "alice" and ref["purposes"][a1] == "receive"
    assert w2.mnemonic() == w.mnemonic()
    assert w2.dump_privkey(a1) == w.dump_privkey(a1) and w2.dump_privkey(a2) == w.dump_privkey(a2)
    assert w2.labels[core.hash160(core.secp_pubkey_create(w.keys[w.pool[0]][0], True))] == "" and w2.pool == w.pool
    for _ in range(5):  # pool first, then the chain continues where the exported wallet stands
        assert w2.new_address("x") == w.new_address("x")


def test_export_legacy_hd_wallet_round_trips(core, tmp_path):
    """-bip44=0 (the 0.15 layout): the seed becomes a wallet key of keypath "s" named by the HD
    chain, and the chain continues at the same m/0'/0'/i'."""
    from nodexa_chain_core_amd.wallet.wallet import Wallet
    from nodexa_chain_core_amd.wallet.walletdb import read_wallet_dat

    params = _params()
    w = Wallet(None, params, str(tmp_path / "w.json"), bip44=False)
    a = [w.new_address("l%d" % i) for i in range(3)]
    w2, dat = _export_reimport(core, params, w, tmp_path)
    ref = read_wallet_dat(dat)
    spub = core.secp_pubkey_create(w.hd["seed"], True)
    assert ref["hdchain"]["version"] == 2 and ref["hdchain"]["seed_id"] == core.hash160(spub)
    assert ref["keymeta"][spub]["hdkeypath"] == "s"
    assert [w2.dump_privkey(x) for x in a] == [w.dump_privkey(x) for x in a]
    assert w2.new_address("y") == w.new_address("y")


def test_export_encrypted_wallet_round_trips(core, tmp_path):
    """An encrypted wallet exports its master key and encrypted secrets as they are and its BIP39
    data in the reference's form (EncryptBip39: IV = word hash); locked, a wallet made here refuses
    (its BIP39 data is held in this node's form); the import unlocks with the same passphrase."""
    from nodexa_chain_core_amd.wallet.wallet import Wallet, WalletError
    from nodexa_chain_core_amd.wallet.walletdb import read_wallet_dat, write_wallet_dat

    params = _params()
    w = Wallet(None, params, str(tmp_path / "w.json"))
    a1 = w.new_address("a")
    words = w.mnemonic()
    wif = w.dump_privkey(a1)
    w.encrypt("pw one")
    with pytest.raises(WalletError, match="passphrase"):
        write_wallet_dat(w, str(tmp_path / "locked.dat"))
    w.unlock("pw one")
    w2, dat = _export_reimport(core, params, w, tmp_path)
    ref = read_wallet_dat(dat)
    assert ref["mkeys"] and not ref["keys"] and len(ref["ckeys"]) == len(w.keys)
    assert {"cbip39words", "cbip39vchseed"} <= set(ref["bip39"]) and "bip39words" not in ref["bip39"]
    assert w2.locked
    w2.unlock("pw one")
    assert w2.dump_privkey(a1) == wif and w2.mnemonic() == words
    # once imported, the reference form is kept: the imported wallet exports again while locked
    w2.lock_wallet()
    w3, _ = _export_reimport(core, params, w2, tmp_path, "again.dat")
    w3.unlock("pw one")
    assert w3.dump_privkey(a1) == wif and w3.mnemonic() == words


@needs_libdb
def test_reference_fixture_survives_import_export(core, tmp_path):
    """A wallet.dat in the reference's layout (written by libdb) -> import -> export -> import: the
    keys, labels, pool, scripts and HD chain come through unchanged."""
    from nodexa_chain_core_amd.wallet import bip39
    from nodexa_chain_core_amd.wallet.wallet import Wallet

    params = _params()
    words = bip39.generate(128)
    recs, secrets, seed = _bip44_wallet_records(core, words, "pp", 3)
    a0 = _p2pkh_addr(core, params, secrets[0])
    recs.append((rkey("name", vec(a0.encode())), vec(b"savings")))
    recs.append(pool_record(1, core.secp_pubkey_create(secrets[2], True)))
    redeem = b"\x51\x21" + core.secp_pubkey_create(secrets[1], True) + b"\x51\xae"
    recs.append((rkey("cscript", core.hash160(redeem)), vec(redeem)))
    dat = str(tmp_path / "wallet.dat")
    bdb_write(dat, recs)
    w = Wallet(None, params, str(tmp_path / "w.json"), import_from=dat)
    w2, _ = _export_reimport(core, params, w, tmp_path)
    assert w2.mnemonic() == (words, "pp") and w2.dump_privkey(a0) == w.dump_privkey(a0)
    assert w2.labels[core.hash160(core.secp_pubkey_create(secrets[0], True))] == "savings"
    assert w2.pool == w.pool and w2.redeem_scripts == w.redeem_scripts
    assert w2.new_address("z") == w.new_address("z")


def test_backupwallet_writes_reference_wallet_dat(core, node_factory, tmp_path):  # noqa: F811
    """backupwallet to a .dat name: a wallet.dat in the reference's format holding the node's keys."""
    from nodexa_chain_core_amd.wallet.walletdb import read_wallet_dat

    node, addr = node_factory()
    c = client(node)
    a = c.getnewaddress("backup-label")
    dest = str(tmp_path / "backup.dat")
    c.backupwallet(dest)
    ref = read_wallet_dat(dest)
    assert ref["names"][a] == "backup-label" and ref["hdchain"] is not None
    w = node.wallets[next(iter(node.wallets))] if hasattr(node, "wallets") else node.wallet
    assert len(ref["keys"]) == len(w.keys)
    c.backupwallet(str(tmp_path / "backup.json"))  # any other name: the JSON wallet
    assert open(tmp_path / "backup.json").read().lstrip().startswith("{")
