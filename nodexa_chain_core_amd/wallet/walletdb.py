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
