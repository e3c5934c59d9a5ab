"""Import of a reference wallet.dat (Berkeley DB) into this node's JSON wallet.

The reference stores its wallet as Berkeley DB btree records in the sub-database "main" of
wallet.dat (src/wallet/db.cpp), one record per (type, id) key, parsed by ReadKeyValue
(src/wallet/walletdb.cpp:244-590). This node keeps wallets as JSON (wallet/wallet.py); a datadir
that holds a reference wallet.dat and no JSON wallet of that name is imported once at start-up
(node.py) — read-only, the .dat file is left as it is. The pages are walked natively
(csrc/store/bdb.cpp, `_core.bdb_read`); the records are the reference's serializations:

  key      ("key", CPubKey)       -> CPrivKey (DER, src/key.cpp:69-120) [+ sha256d(pub || privkey)]
  wkey     ("wkey", CPubKey)      -> CWalletKey (CPrivKey, created, expires, comment)
  ckey     ("ckey", CPubKey)      -> AES-256-CBC(master, IV = sha256d(pub)[:16]) of the secret
  mkey     ("mkey", u32 id)       -> CMasterKey (crypted key, salt, method, iterations, params)
  name     ("name", address)      -> label;  purpose ("purpose", address) -> purpose
  keymeta  ("keymeta", CPubKey)   -> CKeyMetadata (version, created, [hdKeypath, seed id])
  pool     ("pool", i64 index)    -> CKeyPool (version, time, CPubKey, [internal])
  hdchain  "hdchain"              -> CHDChain (version, external counter, seed id, [internal
                                     counter], [bip44 flag]; src/wallet/walletdb.h:62-119)
  bip39words / bip39passphrase / bip39vchseed (and their "c" encrypted forms, IV = the word
                                     hash stored with the words; src/wallet/crypter.cpp:352-413)
  cscript  ("cscript", hash160)   -> redeem script;  watchs ("watchs", script) -> '1'
  tx, acentry, destdata, orderposnext, defaultkey, version, minversion: not imported (the
                                     transaction history is rebuilt by a rescan of the chain)

Keys are imported when their public key is compressed (every key a reference wallet has created
since 0.6); an uncompressed key is counted in the report and left out, since this wallet's key
store, WIF encoding and signers are compressed-key only.
"""
from __future__ import annotations

import struct

from .. import core

_core = core()

BDB_BTREE_MAGIC = 0x053162


def is_bdb_file(path: str) -> bool:
    """A Berkeley DB btree file (magic at byte 12, either byte order)."""
    try:
        with open(path, "rb") as f:
            head = f.read(16)
    except OSError:
        return False
    if len(head) < 16:
        return False
    m = struct.unpack_from("<I", head, 12)[0]
    return m == BDB_BTREE_MAGIC or m == struct.unpack(">I", struct.pack("<I", BDB_BTREE_MAGIC))[0]


class _Stream:
    """CDataStream reads: compact sizes, vectors / strings, little-endian integers."""

    def __init__(self, b: bytes):
        self.b, self.i = b, 0

    def take(self, n: int) -> bytes:
        if self.i + n > len(self.b):
            raise ValueError("record truncated")
        out = self.b[self.i:self.i + n]
        self.i += n
        return out

    def compact(self) -> int:
        n = self.take(1)[0]
        if n < 253:
            return n
        return int.from_bytes(self.take({253: 2, 254: 4, 255: 8}[n]), "little")

    def vec(self) -> bytes:
        return self.take(self.compact())

    def u32(self) -> int:
        return struct.unpack("<I", self.take(4))[0]

    def i32(self) -> int:
        return struct.unpack("<i", self.take(4))[0]

    def i64(self) -> int:
        return struct.unpack("<q", self.take(8))[0]

    def boolean(self) -> bool:
        return self.take(1)[0] != 0

    def left(self) -> int:
        return len(self.b) - self.i


def privkey_from_der(der: bytes) -> bytes:
    """The 32-byte secret of a CPrivKey (the DER ECPrivateKey of ec_privkey_export_der:
    SEQUENCE { INTEGER 1, OCTET STRING secret, ... })."""
    s = _Stream(der)
    if s.take(1) != b"\x30":
        raise ValueError("CPrivKey: not a DER sequence")
    n = s.take(1)[0]
    if n & 0x80:
        s.take(n & 0x7F)
    if s.take(3) != b"\x02\x01\x01" or s.take(1) != b"\x04":
        raise ValueError("CPrivKey: unexpected DER layout")
    ln = s.take(1)[0]
    if not 1 <= ln <= 32:
        raise ValueError("CPrivKey: bad secret length")
    secret = s.take(ln).rjust(32, b"\x00")
    if not _core.secp_seckey_valid(secret):
        raise ValueError("CPrivKey: secret out of range")
    return secret


def read_wallet_dat(path: str) -> dict:
    """Parse the records of a reference wallet.dat into plain Python values (see the module
    docstring). Raises ValueError / RuntimeError on a corrupt file, as LoadWallet fails on one."""
    out = {"keys": {}, "ckeys": {}, "mkeys": {}, "names": {}, "purposes": {}, "keymeta": {}, "pool": {},
           "hdchain": None, "bip39": {}, "cscripts": {}, "watchs": [], "version": None, "skipped": {}}
    for kb, vb in _core.bdb_read(path, "main"):
        k, v = _Stream(kb), _Stream(vb)
        t = k.vec().decode("latin-1")
        if t in ("key", "wkey"):
            pub = k.vec()
            if t == "key":
                der = v.vec()
            else:
                v.i32()  # CWalletKey: the serialization version precedes vchPrivKey
                der = v.vec()
            secret = privkey_from_der(der)
            if t == "key" and v.left() >= 32:
                h = v.take(32)
                if h != bytes(32) and _core.sha256d(pub + der) != h:
                    raise ValueError("Error reading wallet database: CPubKey/CPrivKey corrupt")
            if _core.secp_pubkey_create(secret, len(pub) == 33) != pub:
                raise ValueError("Error reading wallet database: CPrivKey corrupt")
            out["keys"][pub] = secret
        elif t == "ckey":
            out["ckeys"][k.vec()] = v.vec()
        elif t == "mkey":
            nid = k.u32()
            if nid in out["mkeys"]:
                raise ValueError(f"Error reading wallet database: duplicate CMasterKey id {nid}")
            out["mkeys"][nid] = {"crypted": v.vec(), "salt": v.vec(), "method": v.u32(), "rounds": v.u32(),
                                 "other": v.vec()}
        elif t in ("name", "purpose"):
            out[t + "s"][k.vec().decode()] = v.vec().decode()
        elif t == "keymeta":
            pub = k.vec()
            ver, created = v.i32(), v.i64()
            path_, seed = "", None
            if ver >= 10:  # CKeyMetadata::VERSION_WITH_HDDATA
                path_, seed = v.vec().decode(), v.take(20)
            out["keymeta"][pub] = {"created": created, "hdkeypath": path_, "seed_id": seed}
        elif t == "pool":
            idx = k.i64()
            v.i32()  # client version
            tm, pub = v.i64(), v.vec()
            out["pool"][idx] = {"time": tm, "pub": pub, "internal": v.boolean() if v.left() else False}
        elif t == "hdchain":
            ver, ext = v.i32(), v.u32()
            seed_id = v.take(20)
            internal = v.u32() if ver >= 2 else 0
            bip44 = v.boolean() if ver == 3 else False
            out["hdchain"] = {"version": ver, "external": ext, "internal": internal, "seed_id": seed_id,
                              "bip44": bip44}
        elif t in ("bip39words", "cbip39words"):
            out["bip39"][t] = (v.take(32), v.vec())
        elif t in ("bip39passphrase", "cbip39passphrase", "bip39vchseed", "cbip39vchseed"):
            out["bip39"][t] = v.vec()
        elif t == "cscript":
            out["cscripts"][k.take(20)] = v.vec()
        elif t == "watchs":
            script = k.vec()
            if v.take(1) == b"1":
                out["watchs"].append(script)
        elif t == "version":
            out["version"] = v.i32()
        else:
            out["skipped"][t] = out["skipped"].get(t, 0) + 1
    return out


# ---------------------------------------------------------------------------------------- export
# The reference's CLIENT_VERSION (configure.ac: 4.4.4.2) and the wallet feature level it writes
# (FEATURE_LATEST = FEATURE_COMPRPUBKEY, src/wallet/wallet.h:94-105).
CLIENT_VERSION = 4_04_04_02
FEATURE_LATEST = 10000
_SECP_P = (1 << 256) - (1 << 32) - 977
_SECP_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
_SECP_GX = bytes.fromhex("79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798")
_SECP_GY = bytes.fromhex("483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8")


def _cs(n: int) -> bytes:
    if n < 253:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + struct.pack("<H", n)
    if n <= 0xFFFFFFFF:
        return b"\xfe" + struct.pack("<I", n)
    return b"\xff" + struct.pack("<Q", n)


def _vec(b: bytes) -> bytes:
    return _cs(len(b)) + b


def _rkey(t: str, *parts: bytes) -> bytes:
    return _vec(t.encode()) + b"".join(parts)


def privkey_to_der(secret: bytes, pub: bytes) -> bytes:
    """CPrivKey: SEC1 ECPrivateKey with the explicit secp256k1 parameters, as ec_privkey_export_der
    writes it (src/key.cpp:66-120): 214 bytes for a compressed key, 279 for an uncompressed one
    (the generator and the public key in the form of the key)."""
    comp = len(pub) == 33
    g = (b"\x02" + _SECP_GX) if comp else (b"\x04" + _SECP_GX + _SECP_GY)
    curve = (b"\x30\x2c\x06\x07\x2a\x86\x48\xce\x3d\x01\x01\x02\x21\x00" + _SECP_P.to_bytes(32, "big")
             + b"\x30\x06\x04\x01\x00\x04\x01\x07" + bytes([0x04, len(g)]) + g
             + b"\x02\x21\x00" + _SECP_N.to_bytes(32, "big") + b"\x02\x01\x01")
    params = b"\x02\x01\x01" + curve

    def der_len(n: int) -> bytes:
        return bytes([n]) if n < 0x80 else (b"\x81" + bytes([n]) if n < 0x100 else b"\x82" + n.to_bytes(2, "big"))

    seq = b"\x30" + der_len(len(params)) + params
    tagged = b"\xa0" + der_len(len(seq)) + seq
    bits = b"\x03" + der_len(len(pub) + 1) + b"\x00" + pub
    body = b"\x02\x01\x01\x04\x20" + secret + tagged + b"\xa1" + der_len(len(bits)) + bits
    return b"\x30" + der_len(len(body)) + body


def _internal_path(path: str) -> bool:
    """A change-chain keypath: m/44'/coin'/account'/1/i (BIP44) or m/0'/1'/i' (the 0.15 layout)."""
    parts = path.split("/")
    if len(parts) == 6 and parts[1] == "44'":
        return parts[4] == "1"
    return len(parts) == 4 and parts[2] == "1'"


def _keymeta(created: int, path: str, seed_id: bytes) -> bytes:
    # CKeyMetadata VERSION_WITH_HDDATA: version, created, hdKeypath, hd_seed_id (walletdb.h:124-152)
    return struct.pack("<iq", 10, int(created)) + _vec(path.encode()) + seed_id


def wallet_dat_records(w) -> list[tuple[bytes, bytes]]:
    """The reference's wallet.dat records of wallet `w` (wallet/wallet.Wallet): the inverse of
    read_wallet_dat. Plain wallets: key + keymeta per key, name / purpose for the receiving
    addresses handed out, the keypool, the HD chain (CHDChain v3 with the BIP39 words, passphrase
    and seed; the 0.15 layout: v2 with the seed as a key of path "s"), redeem and watch-only
    scripts, version / minversion. Encrypted wallets: mkey + ckey (the same CCrypter blobs this
    wallet keeps) and the cbip39 forms; they need the wallet unlocked when its BIP39 data or seed
    is not held in the reference's form. Uncompressed keys kept aside by an import go back as the
    records they came from. No transactions: the reference rescans the chain for them."""
    from .wallet import WalletError, _iv

    sha = _core.sha256d
    recs: dict[bytes, bytes] = {}
    crypted = w.mkey is not None
    if crypted and w.locked:
        hd = w.hd or {}
        ref_form = hd.get("ref_words_crypted") and hd.get("ref_word_hash") if hd.get("bip44") else \
            hd.get("master_id") in w.keys
        if hd and not ref_form:  # BIP39 data / seed not held in the reference's encrypted form
            raise WalletError("Error: Please enter the wallet passphrase with walletpassphrase first.")
    master = getattr(w, "_master", None)

    def enc(iv16: bytes, plain: bytes) -> bytes:
        return _core.aes256_cbc_encrypt(master, iv16, plain)

    # HD chain first: it decides the seed id every derived key's metadata carries
    seed_id = bytes(20)
    hd = w.hd
    if hd is not None:
        nxt = hd.get("next", {})
        ext, internal = int(nxt.get("0", 0)), int(nxt.get("1", 0))
        if hd.get("bip44"):
            # CPubKey(64-byte BIP39 seed) is invalid, so the reference's seed_id is Hash160 of nothing
            # (wallet.cpp GenerateNewSeed); derivation reads the seed itself
            seed_id = _core.hash160(b"")
            recs[_rkey("hdchain")] = struct.pack("<iI", 3, ext) + seed_id + struct.pack("<I", internal) + b"\x01"
            if not crypted:
                words = (hd.get("mnemonic") or "").encode()
                recs[_rkey("bip39words")] = sha(words) + _vec(words)
                recs[_rkey("bip39passphrase")] = _vec((hd.get("mnemonic_passphrase") or "").encode())
                recs[_rkey("bip39vchseed")] = _vec(hd["seed"])
            elif hd.get("ref_words_crypted") and hd.get("ref_word_hash"):  # imported: as read
                wh = hd["ref_word_hash"]
                recs[_rkey("cbip39words")] = wh + _vec(hd["ref_words_crypted"])
                if hd.get("ref_pass_crypted"):
                    recs[_rkey("cbip39passphrase")] = _vec(hd["ref_pass_crypted"])
                recs[_rkey("cbip39vchseed")] = _vec(hd["seed_crypted"])
            else:  # EncryptBip39: IV = the first 16 bytes of the word hash (crypter.cpp:352-384)
                words = (hd.get("mnemonic") or "").encode()
                wh = sha(words)
                recs[_rkey("cbip39words")] = wh + _vec(enc(wh[:16], words))
                pp = (hd.get("mnemonic_passphrase") or "").encode()
                if pp:
                    recs[_rkey("cbip39passphrase")] = _vec(enc(wh[:16], pp))
                recs[_rkey("cbip39vchseed")] = _vec(enc(wh[:16], hd["seed"]))
        else:
            # the 0.15 layout: the seed is a wallet key (DeriveNewSeed, keypath "s"); an imported
            # wallet already holds it among its keys (its id is the HD chain's), a wallet made here
            # keeps it apart and it is written as that key
            if hd["master_id"] in w.keys:
                seed_id = hd["master_id"]
            else:
                seed = hd.get("seed")
                if seed is None:
                    raise WalletError("Error: Please enter the wallet passphrase with walletpassphrase first.")
                spub = _core.secp_pubkey_create(seed, True)
                seed_id = _core.hash160(spub)
                if crypted:
                    recs[_rkey("ckey", _vec(spub))] = _vec(enc(_iv(spub), seed))
                else:
                    der = privkey_to_der(seed, spub)
                    recs[_rkey("key", _vec(spub))] = _vec(der) + sha(spub + der)
                recs[_rkey("keymeta", _vec(spub))] = _keymeta(0, "s", seed_id)
            recs[_rkey("hdchain")] = struct.pack("<iI", 2, ext) + seed_id + struct.pack("<I", internal)
    pool = set(w.pool)
    for h, (sec, pub) in w.keys.items():
        path = w.hdpath.get(h, "")
        if crypted:
            recs[_rkey("ckey", _vec(pub))] = _vec(w.crypted[h])
        else:
            der = privkey_to_der(sec, pub)
            recs[_rkey("key", _vec(pub))] = _vec(der) + sha(pub + der)
        recs[_rkey("keymeta", _vec(pub))] = _keymeta(w.created.get(h, 0), path, seed_id if path else bytes(20))
        change = w.labels.get(h) == "change" or _internal_path(path)
        if h not in pool and not change and path != "s":
            addr = w.address_of(h).encode()
            recs[_rkey("name", _vec(addr))] = _vec(w.labels.get(h, "").encode())
            recs[_rkey("purpose", _vec(addr))] = _vec(b"receive")
    for i, h in enumerate(w.pool, start=1):
        pub = w.keys[h][1]
        internal = _internal_path(w.hdpath.get(h, ""))
        recs[_rkey("pool", struct.pack("<q", i))] = (struct.pack("<iq", CLIENT_VERSION, w.created.get(h, 0))
                                                     + _vec(pub) + bytes([internal]))
    for pub, rec in getattr(w, "uncompressed", {}).items():
        if "crypted" in rec:
            recs[_rkey("ckey", _vec(pub))] = _vec(rec["crypted"])
        else:
            der = privkey_to_der(rec["sec"], pub)
            recs[_rkey("key", _vec(pub))] = _vec(der) + sha(pub + der)
        recs[_rkey("keymeta", _vec(pub))] = _keymeta(0, "", bytes(20))
    for h, script in w.redeem_scripts.items():
        recs[_rkey("cscript", h)] = _vec(script)
    for spk, meta in w.watch.items():
        recs[_rkey("watchs", _vec(spk))] = b"1"
        recs[_rkey("watchmeta", _vec(spk))] = _keymeta(0, "", bytes(20))
        if meta.get("label"):
            try:
                addr = _core.script_to_address(spk, w.params.pubkey_prefix, w.params.script_prefix)
            except Exception:  # noqa: BLE001 - a non-standard script has no address to label
                addr = None
            if addr:
                recs[_rkey("name", _vec(addr.encode()))] = _vec(meta["label"].encode())
                recs[_rkey("purpose", _vec(addr.encode()))] = _vec(b"receive")
    if crypted:
        mk = w.mkey
        recs[_rkey("mkey", struct.pack("<I", 1))] = (_vec(mk["crypted"]) + _vec(mk["salt"])
                                                     + struct.pack("<II", 0, mk["rounds"]) + _vec(b""))
    recs[_rkey("version")] = struct.pack("<i", CLIENT_VERSION)
    recs[_rkey("minversion")] = struct.pack("<i", FEATURE_LATEST)
    return sorted(recs.items())


def write_wallet_dat(w, path: str) -> int:
    """Wallet `w` as a reference wallet.dat at `path` (csrc/store/bdb.cpp writer, sub-database
    "main"); returns the record count."""
    recs = wallet_dat_records(w)
    _core.bdb_write(path, recs, "main")
    return len(recs)
