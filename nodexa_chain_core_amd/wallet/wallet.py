"""Key wallet (the subset a mining / validating node uses).

Parity (behaviour; a reference wallet.dat is imported once by wallet/walletdb.py): CWallet key store and its RPCs in
src/wallet/rpcwallet.cpp (getnewaddress, getbalance, listunspent, sendtoaddress, sendmany,
dumpprivkey / importprivkey, signrawtransaction, getwalletinfo), CKey::Sign + the standard
signature producers of src/script/sign.cpp for P2PKH, P2PK, P2WPKH and P2SH-P2WPKH outputs, WIF
secrets (base58check: SECRET_KEY prefix, key, 0x01 for compressed keys; src/base58.cpp).

Keys derive from a BIP39 mnemonic along BIP44 paths (or the 0.15 hardened BIP32 layout with
-bip44=0; csrc/crypto/secp256k1.cpp signs with RFC 6979) and live in <datadir>/wallet.json,
written atomically, optionally AES-256-CBC encrypted (encryptwallet). Balances come from the node's UTXO set (CoinsView.outputs_for_scripts) plus the
mempool's unconfirmed outputs to the wallet's scripts.
"""
from __future__ import annotations

import json
import os
import struct
import threading
import time

from .. import core

_core = core()

# base58Prefixes[SECRET_KEY] (src/chainparams.cpp:191, 350, 517)
SECRET_PREFIX = {"main": 112, "test": 114, "regtest": 114}
SIGHASH_ALL = 1
COIN = 100_000_000
DEFAULT_FEE_RATE = 2_000_000  # sat per kvB: above the 0.01 CLORE/kvB min relay fee
DEFAULT_KEYPOOL_SIZE = 100
DEFAULT_TX_CONFIRM_TARGET = 6   # src/wallet/wallet.h:69
DEFAULT_TRANSACTION_MINFEE = 1_000_000  # -mintxfee (src/wallet/wallet.h:57)
DEFAULT_DERIVE_ROUNDS = 25000  # CMasterKey nDeriveIterations default
UNLOCK_NEEDED = "Error: Please enter the wallet passphrase with walletpassphrase first."
HARDENED = 0x80000000
WALLET_INCREMENTAL_RELAY_FEE = 5000  # sat per kB (src/wallet/wallet.h:59)
DEFAULT_DISCARD_FEE = 10_000  # sat per kvB (src/wallet/wallet.h): change worth less than spending it is dropped
DUST_THRESHOLD = 546  # GetDustThreshold of a P2PKH output at DUST_RELAY_TX_FEE (chain/policy.py)
# nExtCoinType (src/chainparams.cpp:196, 355, 522): the BIP44 coin_type level
EXT_COIN_TYPE = {"main": 1313, "test": 1, "regtest": 1}
# base58Prefixes[EXT_SECRET_KEY] (src/chainparams.cpp:193, 352, 519)
EXT_SECRET_PREFIX = {"main": bytes.fromhex("0488ADE4"), "test": bytes.fromhex("04358394"),
                     "regtest": bytes.fromhex("04358394")}


def _iv(pub: bytes) -> bytes:
    """CCrypter IV for a key: the first 16 bytes of sha256d(pubkey) (EncryptSecret)."""
    return _core.sha256d(pub)[:16]


def _bip32_master(seed: bytes) -> tuple[bytes, bytes]:
    i = _core.hmac_sha512(b"Bitcoin seed", seed)
    return i[:32], i[32:]


def _ckd_priv(k: bytes, c: bytes, index: int, hardened: bool = True):
    """BIP32 private child: HMAC-SHA512(c, 0x00 || k || ser32(i | 2^31)) when hardened, else
    HMAC-SHA512(c, serP(k*G) || ser32(i)); child = k + IL. None if the child is invalid."""
    if hardened:
        data = b"\x00" + k + struct.pack(">I", index | HARDENED)
    else:
        data = _core.secp_pubkey_create(k, True) + struct.pack(">I", index)
    i = _core.hmac_sha512(c, data)
    child = _core.secp_seckey_tweak_add(k, i[:32])
    return None if child is None else (child, i[32:])


def ext_key_b58(k: bytes, c: bytes, network: str, depth: int = 0, fingerprint: bytes = b"\0" * 4,
                child: int = 0) -> str:
    """CExtKey::Encode under base58Prefixes[EXT_SECRET_KEY] (xprv / tprv)."""
    version = EXT_SECRET_PREFIX[network]
    return _core.base58check_encode(version + bytes([depth]) + fingerprint + struct.pack(">I", child) + c
                                    + b"\x00" + k)


def _push(d: bytes) -> bytes:
    return _core.script_push_data(d)


def p2pkh(h160: bytes) -> bytes:
    return b"\x76\xa9\x14" + h160 + b"\x88\xac"


class WalletError(Exception):
    pass


def _pushes(script: bytes) -> list[bytes]:
    """Data of each push of a push-only script (OP_0 as b"")."""
    out, i = [], 0
    while i < len(script):
        op = script[i]
        i += 1
        if op == 0:
            out.append(b"")
            continue
        if op < 0x4C:
            n = op
        elif op == 0x4C:
            n = script[i]
            i += 1
        elif op == 0x4D:
            n = int.from_bytes(script[i:i + 2], "little")
            i += 2
        else:
            break
        out.append(script[i:i + n])
        i += n
    return out


def parse_multisig(script: bytes):
    """OP_m <pubkey>... OP_n OP_CHECKMULTISIG -> (m, [pubkeys]) or None."""
    if len(script) < 3 or script[-1] != 0xAE or not (0x51 <= script[0] <= 0x60) or not (0x51 <= script[-2] <= 0x60):
        return None
    m, n = script[0] - 0x50, script[-2] - 0x50
    pubs = _pushes(script[1:-2])
    if len(pubs) != n or m > n or any(len(p) not in (33, 65) for p in pubs):
        return None
    return m, pubs


def multisig_script(m: int, pubkeys: list[bytes]) -> bytes:
    return bytes([0x50 + m]) + b"".join(_push(p) for p in pubkeys) + bytes([0x50 + len(pubkeys), 0xAE])


class Wallet:
    def __init__(self, state, params, path: str | None, bip44: bool = True, mnemonic: str = "",
                 mnemonic_passphrase: str = "", import_from: str | None = None, keep_uncompressed: bool = False):
        self.state = state
        self.params = params
        self.path = path
        self.lock = threading.RLock()
        self.keys: dict[bytes, tuple[bytes, bytes]] = {}  # hash160(pubkey) -> (secret, compressed pubkey)
        self.labels: dict[bytes, str] = {}
        self.created: dict[bytes, int] = {}
        self._p2sh_wpkh: dict[bytes, bytes] = {}  # hash160(0x0014 || h) -> h
        self.redeem_scripts: dict[bytes, bytes] = {}  # hash160(script) -> script (addmultisigaddress)
        self.watch: dict[bytes, dict] = {}  # watch-only scriptPubKey -> {"label", "solvable"} (importaddress)
        self.walletrbf = False  # -walletrbf: sends signal BIP125 replaceability (DEFAULT_WALLET_RBF)
        self.history = None    # wallet/history.WalletHistory, attached by the node
        self.pay_tx_fee = 0               # settxfee / -paytxfee (sat per kvB; 0 = use fee estimation)
        self.fallback_fee = DEFAULT_FEE_RATE  # -fallbackfee: used while the estimator has no answer
        self.tx_confirm_target = DEFAULT_TX_CONFIRM_TARGET  # -txconfirmtarget
        self.min_tx_fee = DEFAULT_TRANSACTION_MINFEE  # -mintxfee (sat per kvB)
        self.max_tx_fee: int | None = None            # -maxtxfee cap on one transaction's fee (None: node's)
        self.keypool_size = DEFAULT_KEYPOOL_SIZE      # -keypool
        self.broadcast = True                         # -walletbroadcast
        self.spend_zeroconf_change = True             # -spendzeroconfchange (DEFAULT_SPEND_ZEROCONF_CHANGE)
        self.discard_fee = DEFAULT_DISCARD_FEE        # -discardfee (sat per kvB)
        self.reject_long_chains = False               # -walletrejectlongchains
        self.hdpath: dict[bytes, str] = {}      # hdkeypath of derived keys
        self.pool: list[bytes] = []             # keypool: reserved keys not yet handed out
        self.hd: dict | None = None             # {"master_id", "next", "seed", "seed_crypted"}
        self.crypted: dict[bytes, bytes] = {}   # encrypted secrets (encryptwallet)
        self.mkey: dict | None = None           # {"salt", "rounds", "crypted"} master key record
        self._master: bytes | None = None       # the master key while unlocked
        self._relock = None
        self.unlocked_until = 0
        self.import_report: dict | None = None  # what import_from brought in (walletdb.py)
        # uncompressed keys of an imported wallet.dat (pub -> secret or encrypted blob): this wallet
        # does not spend with them yet, so they are kept verbatim in the saved file, not dropped
        self.uncompressed: dict[bytes, dict] = {}
        self._keep_uncompressed = keep_uncompressed
        if path and os.path.exists(path):
            self._load()
        elif import_from:
            self.import_report = self._import_reference(import_from)
        if self.hd is None and not self.keys:  # a new wallet is HD (CWallet::GenerateNewSeed)
            self._init_hd(bip44, mnemonic, mnemonic_passphrase)

    # ------------------------------------------------------------------ persistence

    @property
    def fee_rate(self) -> int:
        """GetMinimumFee's feerate (src/wallet/fees.cpp): -paytxfee / settxfee when set, else the
        node's estimatesmartfee at -txconfirmtarget (economical when the wallet signals BIP125),
        else -fallbackfee; never below -mintxfee or the min relay fee."""
        rate = self.pay_tx_fee
        if not rate:
            est = getattr(self.state, "fee_estimator", None) if self.state is not None else None
            if est is not None:
                rate, _, _, _ = est.estimate_smart_fee(self.tx_confirm_target, not self.walletrbf)
            rate = rate or self.fallback_fee
        floor = max(self.min_tx_fee, getattr(self.state, "min_relay_fee", 0) if self.state else 0)
        return max(rate, floor)

    @fee_rate.setter
    def fee_rate(self, v: int) -> None:
        self.pay_tx_fee = int(v)

    def _load(self) -> None:
        with open(self.path) as f:
            data = json.load(f)
        for rec in data.get("uncompressed_keys", []):
            self.uncompressed[bytes.fromhex(rec["pub"])] = {k: bytes.fromhex(v) for k, v in rec.items() if k != "pub"}
        mk = data.get("mkey")
        if mk:
            self.mkey = {"salt": bytes.fromhex(mk["salt"]), "rounds": int(mk["rounds"]),
                         "crypted": bytes.fromhex(mk["crypted"])}
        for k in data.get("keys", []):
            if "wif" in k:
                h = self._add_secret(self.decode_wif(k["wif"]), k.get("label", ""), k.get("created", 0), save=False)
            else:
                pub = bytes.fromhex(k["pub"])
                h = _core.hash160(pub)
                self.keys[h] = (None, pub)
                self.crypted[h] = bytes.fromhex(k["crypted"])
                self._p2sh_wpkh[_core.hash160(b"\x00\x14" + h)] = h
                self.labels[h] = k.get("label", "")
                self.created[h] = k.get("created", 0)
            if k.get("hdkeypath"):
                self.hdpath[h] = k["hdkeypath"]
            if k.get("pool"):
                self.pool.append(h)
        hd = data.get("hd")
        if hd:
            self.hd = {"master_id": bytes.fromhex(hd["master_id"]), "next": dict(hd["next"]),
                       "seed": bytes.fromhex(hd["seed"]) if hd.get("seed") else None,
                       "seed_crypted": bytes.fromhex(hd["seed_crypted"]) if hd.get("seed_crypted") else None,
                       "bip44": bool(hd.get("bip44", False)), "mnemonic": hd.get("mnemonic"),
                       "mnemonic_passphrase": hd.get("mnemonic_passphrase"),
                       "mnemonic_crypted": bytes.fromhex(hd["mnemonic_crypted"]) if hd.get("mnemonic_crypted")
                       else None}
            for f in ("seed_iv", "ref_words_crypted", "ref_pass_crypted", "ref_word_hash"):  # an imported wallet.dat's
                if hd.get(f) is not None:
                    self.hd[f] = bytes.fromhex(hd[f])
        for rs in data.get("redeem_scripts", []):
            script = bytes.fromhex(rs)
            self.redeem_scripts[_core.hash160(script)] = script
        for wo in data.get("watch", []):
            self.watch[bytes.fromhex(wo["spk"])] = {"label": wo.get("label", ""), "solvable": wo.get("solvable", False)}

    def _import_reference(self, dat_path: str) -> dict:
        """A reference wallet.dat (wallet/walletdb.py) as this wallet: keys (plain or encrypted with
        the reference's master key, which encrypts the same way, CCrypter), labels, key metadata,
        the keypool, the HD chain with its counters and BIP39 data, redeem scripts and watch-only
        scripts. Saved as JSON at once; the .dat file is only read."""
        from .walletdb import read_wallet_dat

        ref = read_wallet_dat(dat_path)
        report = {"keys": 0, "crypted_keys": 0, "uncompressed_skipped": 0, "labels": 0, "pool": 0,
                  "scripts": len(ref["cscripts"]), "watch": len(ref["watchs"]), "hd": None,
                  "encrypted": bool(ref["mkeys"]), "version": ref["version"], "not_imported": ref["skipped"]}
        if ref["mkeys"]:
            mk = ref["mkeys"][min(ref["mkeys"])]  # CWallet::Unlock tries each; one is all encryptwallet writes
            if mk["method"] != 0:
                raise WalletError(f"wallet.dat master key derivation method {mk['method']} is not supported")
            self.mkey = {"salt": mk["salt"], "rounds": mk["rounds"], "crypted": mk["crypted"]}
        pubs: dict[bytes, bytes] = {}  # hash160 -> pub of every imported key
        unc = {pub: {"sec": sec} for pub, sec in ref["keys"].items() if len(pub) != 33}
        unc.update({pub: {"crypted": blob} for pub, blob in ref["ckeys"].items() if len(pub) != 33})
        if unc and not self._keep_uncompressed:
            # funds at those keys' addresses would drop out of this wallet: refuse, unless asked
            raise WalletError(f"wallet.dat holds {len(unc)} uncompressed key(s), which this wallet cannot spend "
                              "with yet; -walletkeepuncompressed=1 imports the rest and keeps them aside "
                              "(saved verbatim, not spendable here)")
        self.uncompressed = unc
        for pub, sec in ref["keys"].items():
            if len(pub) != 33:
                report["uncompressed_skipped"] += 1
                continue
            h = _core.hash160(pub)
            self.keys[h] = (None if self.mkey is not None else sec, pub)
            if self.mkey is not None:  # a plain key in an encrypted wallet (written before encryption)
                raise WalletError("wallet.dat holds unencrypted keys beside a master key")
            pubs[h] = pub
            report["keys"] += 1
        for pub, blob in ref["ckeys"].items():
            if len(pub) != 33:
                report["uncompressed_skipped"] += 1
                continue
            if self.mkey is None:
                raise WalletError("wallet.dat holds encrypted keys but no master key")
            h = _core.hash160(pub)
            self.keys[h] = (None, pub)
            self.crypted[h] = blob
            pubs[h] = pub
            report["crypted_keys"] += 1
        for h in pubs:
            self._p2sh_wpkh[_core.hash160(b"\x00\x14" + h)] = h
            self.labels.setdefault(h, "")
            self.created.setdefault(h, 0)
        for pub, meta in ref["keymeta"].items():
            h = _core.hash160(pub)
            if h in pubs:
                self.created[h] = meta["created"]
                if meta["hdkeypath"] and meta["hdkeypath"] != "m":
                    self.hdpath[h] = meta["hdkeypath"]
        spk_label: dict[bytes, str] = {}
        for addr, label in ref["names"].items():
            spk = _core.address_to_script(addr, self.params.pubkey_prefix, self.params.script_prefix)
            if spk is None:
                continue
            spk_label[bytes(spk)] = label
            if len(spk) == 25 and spk[3:23] in pubs:
                self.labels[spk[3:23]] = label
                report["labels"] += 1
        for idx in sorted(ref["pool"]):
            h = _core.hash160(ref["pool"][idx]["pub"])
            if h in pubs and h not in self.pool:
                self.pool.append(h)
                report["pool"] += 1
        for h, script in ref["cscripts"].items():
            self.redeem_scripts[_core.hash160(script)] = script
        for script in ref["watchs"]:
            self.watch[script] = {"label": spk_label.get(script, ""), "solvable": False}
        hc = ref["hdchain"]
        if hc is not None and hc["seed_id"] != bytes(20):
            b39 = ref["bip39"]
            hd = {"master_id": hc["seed_id"], "next": {"0": hc["external"], "1": hc["internal"]},
                  "seed": None, "seed_crypted": None, "bip44": hc["bip44"], "mnemonic": None,
                  "mnemonic_passphrase": None, "mnemonic_crypted": None}
            if hc["bip44"]:  # the BIP39 seed (g_vchSeed) and words, IV = the word hash
                if "bip39vchseed" in b39:
                    hd["seed"] = b39["bip39vchseed"]
                    hd["mnemonic"] = b39["bip39words"][1].decode() if "bip39words" in b39 else None
                    hd["mnemonic_passphrase"] = b39.get("bip39passphrase", b"").decode()
                elif "cbip39vchseed" in b39 and "cbip39words" in b39:
                    word_hash, words_c = b39["cbip39words"]
                    hd["seed_crypted"] = b39["cbip39vchseed"]
                    hd["seed_iv"] = word_hash[:16]
                    hd["ref_word_hash"] = word_hash  # kept whole: a wallet.dat export writes it back
                    hd["ref_words_crypted"] = words_c
                    hd["ref_pass_crypted"] = b39.get("cbip39passphrase", b"")
                else:
                    raise WalletError("wallet.dat: a BIP44 HD chain without its BIP39 seed")
            else:  # the 0.15 layout: the seed is the wallet key whose hash160 is the seed id
                if hc["seed_id"] not in pubs:
                    raise WalletError("wallet.dat: HD seed key not found")
                if self.mkey is None:
                    hd["seed"] = self.keys[hc["seed_id"]][0]
                else:
                    hd["seed_crypted"] = self.crypted[hc["seed_id"]]
                    hd["seed_iv"] = _iv(pubs[hc["seed_id"]])
            self.hd = hd
            report["hd"] = {"bip44": hc["bip44"], "external": hc["external"], "internal": hc["internal"]}
        self._save()
        return report

    def _save(self) -> None:
        if not self.path:
            return
        keys = []
        for h, (sec, pub) in self.keys.items():
            e = {"label": self.labels.get(h, ""), "created": self.created.get(h, 0)}
            if self.mkey is not None:
                e.update({"pub": pub.hex(), "crypted": self.crypted[h].hex()})
            else:
                e["wif"] = self.encode_wif(sec)
            if h in self.hdpath:
                e["hdkeypath"] = self.hdpath[h]
            if h in self.pool:
                e["pool"] = True
            keys.append(e)
        data = {"version": 2, "network": self.params.network_id, "keys": keys,
                "redeem_scripts": [rs.hex() for rs in self.redeem_scripts.values()],
                "watch": [{"spk": k.hex(), **v} for k, v in self.watch.items()]}
        if self.hd is not None:
            plain = self.mkey is None
            data["hd"] = {"master_id": self.hd["master_id"].hex(), "next": self.hd["next"],
                          "seed": self.hd["seed"].hex() if self.hd["seed"] is not None and plain else None,
                          "seed_crypted": self.hd["seed_crypted"].hex() if self.hd.get("seed_crypted") else None,
                          "bip44": self.hd.get("bip44", False),
                          "mnemonic": self.hd.get("mnemonic") if plain else None,
                          "mnemonic_passphrase": self.hd.get("mnemonic_passphrase") if plain else None,
                          "mnemonic_crypted": self.hd["mnemonic_crypted"].hex() if self.hd.get("mnemonic_crypted")
                          else None}
            for f in ("seed_iv", "ref_words_crypted", "ref_pass_crypted", "ref_word_hash"):
                if self.hd.get(f) is not None:
                    data["hd"][f] = self.hd[f].hex()
        if self.mkey is not None:
            data["mkey"] = {"salt": self.mkey["salt"].hex(), "rounds": self.mkey["rounds"],
                            "crypted": self.mkey["crypted"].hex()}
        if self.uncompressed:  # kept aside from an imported wallet.dat (not spendable here)
            data["uncompressed_keys"] = [{"pub": pub.hex(), **{k: v.hex() for k, v in rec.items()}}
                                         for pub, rec in self.uncompressed.items()]
        tmp = self.path + ".new"
        with open(tmp, "w") as f:
            json.dump(data, f, indent=1)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.path)

    # ------------------------------------------------------------------ keys
    def encode_wif(self, secret: bytes) -> str:
        return _core.base58check_encode(bytes([SECRET_PREFIX[self.params.network_id]]) + secret + b"\x01")

    def decode_wif(self, wif: str) -> bytes:
        raw = _core.base58check_decode(wif)
        if raw is None or raw[0] != SECRET_PREFIX[self.params.network_id] or len(raw) not in (33, 34):
            raise WalletError("Invalid private key encoding")
        secret = raw[1:33]
        if not _core.secp_seckey_valid(secret):
            raise WalletError("Private key outside allowed range")
        return secret

    def _add_secret(self, secret: bytes, label: str = "", created: int | None = None, save: bool = True,
                    hdkeypath: str | None = None) -> bytes:
        pub = _core.secp_pubkey_create(secret, True)
        h = _core.hash160(pub)
        with self.lock:
            self.keys[h] = (secret, pub)
            if self.mkey is not None:
                if self._master is None:
                    raise WalletError(UNLOCK_NEEDED)
                self.crypted[h] = _core.aes256_cbc_encrypt(self._master, _iv(pub), secret)
            self._p2sh_wpkh[_core.hash160(b"\x00\x14" + h)] = h
            self.labels[h] = label
            self.created[h] = int(time.time()) if created is None else created
            if hdkeypath:
                self.hdpath[h] = hdkeypath
            if save:
                self._save()
        return h

    def address_of(self, h160: bytes) -> str:
        return _core.base58check_encode(bytes([self.params.pubkey_prefix]) + h160)

    # ------------------------------------------------------------------ HD chain (BIP32 / BIP39 / BIP44)
    def _init_hd(self, bip44: bool = True, mnemonic: str = "", passphrase: str = "") -> None:
        """GenerateNewSeed. With -bip44 (the default) the seed is the BIP39 seed of a 12-word mnemonic
        (-mnemonic / -mnemonicpassphrase, or freshly generated) and keys derive as
        m/44'/coin'/0'/change/i (CHDChain::SetMnemonic, CWallet::DeriveNewChildKey); with -bip44=0 a
        random 32-byte seed and the 0.15 layout m/0'/0'/i' (receive), m/0'/1'/i' (change)."""
        from . import bip39

        if bip44:
            mnemonic = " ".join(mnemonic.split()) or bip39.generate(128)
            if not bip39.check(mnemonic):
                raise WalletError(f"invalid mnemonic: `{mnemonic}`")
            seed = bip39.to_seed(mnemonic, passphrase)
        else:
            seed = os.urandom(32)
        mk, _ = _bip32_master(seed)
        self.hd = {"master_id": _core.hash160(_core.secp_pubkey_create(mk, True)), "next": {"0": 0, "1": 0},
                   "seed": seed, "seed_crypted": None, "bip44": bip44,
                   "mnemonic": mnemonic if bip44 else None, "mnemonic_passphrase": passphrase if bip44 else None,
                   "mnemonic_crypted": None}

    def mnemonic(self) -> tuple[str, str]:
        """getmywords: (word list, passphrase) of a BIP39 wallet."""
        if self.hd is None or not self.hd.get("bip44"):
            raise WalletError("Error: Wallet doesn't have 12 words. Only new wallets generated by the mnemonic "
                              "phrase will have 12 words")
        if self.hd.get("mnemonic") is None:
            raise WalletError(UNLOCK_NEEDED)
        return self.hd["mnemonic"], self.hd.get("mnemonic_passphrase") or ""

    def _hd_seed(self) -> bytes:
        if self.hd["seed"] is None:
            raise WalletError(UNLOCK_NEEDED)
        return self.hd["seed"]

    def _derive(self, change: bool) -> tuple[bytes, str]:
        chain = "1" if change else "0"
        k, c = _bip32_master(self._hd_seed())
        bip44 = self.hd.get("bip44", False)
        if bip44:
            coin = EXT_COIN_TYPE[self.params.network_id]
            for i, hard in ((44, True), (coin, True), (0, True), (int(chain), False)):
                k, c = _ckd_priv(k, c, i, hard)
        else:
            for i in (0, int(chain)):
                k, c = _ckd_priv(k, c, i)
        while True:
            idx = self.hd["next"][chain]
            self.hd["next"][chain] = idx + 1
            child = _ckd_priv(k, c, idx, not bip44)
            if child is not None:
                path = f"m/44'/{coin}'/0'/{chain}/{idx}" if bip44 else f"m/0'/{chain}'/{idx}'"
                return child[0], path

    def _fresh_key(self, label: str) -> bytes:
        if self.hd is None:
            while True:
                secret = os.urandom(32)
                if _core.secp_seckey_valid(secret):
                    return self._add_secret(secret, label)
        secret, path = self._derive(label == "change")
        return self._add_secret(secret, label, hdkeypath=path)

    def new_address(self, label: str = "") -> str:
        """GetKeyFromPool: a reserved pool key when there is one (works while the wallet is locked),
        else a freshly derived key."""
        with self.lock:
            if self.pool:
                h = self.pool.pop(0)
                self.labels[h] = label
                self._save()
                return self.address_of(h)
            if self.mkey is not None and self._master is None:
                raise WalletError("Error: Keypool ran out, please call keypoolrefill first")
            return self.address_of(self._fresh_key(label))

    def keypool_refill(self, size: int | None = None) -> None:
        size = self.keypool_size if size is None else size
        with self.lock:
            if self.mkey is not None and self._master is None:
                raise WalletError(UNLOCK_NEEDED)
            while len(self.pool) < size:
                self.pool.append(self._fresh_key(""))
            self._save()

    def import_privkey(self, wif: str, label: str = "") -> str:
        return self.address_of(self._add_secret(self.decode_wif(wif), label))

    def dump_privkey(self, address: str) -> str:
        h = self._h160_of(address)
        if h not in self.keys:
            raise WalletError("Private key for address is not known")
        sec = self.keys[h][0]
        if sec is None:
            raise WalletError(UNLOCK_NEEDED)
        return self.encode_wif(sec)

    # ------------------------------------------------------------------ encryption (CCryptoKeyStore)
    @property
    def encrypted(self) -> bool:
        return self.mkey is not None

    @property
    def locked(self) -> bool:
        return self.mkey is not None and self._master is None

    def encrypt(self, passphrase: str, rounds: int = DEFAULT_DERIVE_ROUNDS) -> None:
        """EncryptWallet: a random master key encrypted under the passphrase (BytesToKeySHA512AES),
        every secret and the HD seed encrypted under the master key; the wallet ends up locked."""
        with self.lock:
            if self.mkey is not None:
                raise WalletError("Error: running with an encrypted wallet, but encryptwallet was called.")
            if not passphrase:
                raise WalletError("passphrase can not be empty")
            master = os.urandom(32)
            salt = os.urandom(8)
            key, iv = _core.bytes_to_key_sha512(passphrase, salt, rounds)
            self.mkey = {"salt": salt, "rounds": rounds, "crypted": _core.aes256_cbc_encrypt(key, iv, master)}
            for h, (sec, pub) in self.keys.items():
                self.crypted[h] = _core.aes256_cbc_encrypt(master, _iv(pub), sec)
            if self.hd is not None:
                self.hd["seed_crypted"] = _core.aes256_cbc_encrypt(master, _iv(b"hdseed"), self.hd["seed"])
                if self.hd.get("mnemonic") is not None:
                    words = json.dumps([self.hd["mnemonic"], self.hd.get("mnemonic_passphrase") or ""]).encode()
                    self.hd["mnemonic_crypted"] = _core.aes256_cbc_encrypt(master, _iv(b"bip39words"), words)
            self._master = master
            self.keypool_refill()
            self._save()
            self.lock_wallet()

    def _master_from(self, passphrase: str) -> bytes | None:
        key, iv = _core.bytes_to_key_sha512(passphrase, self.mkey["salt"], self.mkey["rounds"])
        master = _core.aes256_cbc_decrypt(key, iv, self.mkey["crypted"])
        if master is None or len(master) != 32:
            return None
        for h, (_, pub) in list(self.keys.items())[:1]:  # the check CCryptoKeyStore::Unlock does
            sec = _core.aes256_cbc_decrypt(master, _iv(pub), self.crypted[h])
            if sec is None or _core.secp_pubkey_create(sec, True) != pub:
                return None
        return master

    def unlock(self, passphrase: str, timeout: int = 0) -> None:
        with self.lock:
            if self.mkey is None:
                raise WalletError("Error: running with an unencrypted wallet, but walletpassphrase was called.")
            master = self._master_from(passphrase)
            if master is None:
                raise WalletError("Error: The wallet passphrase entered was incorrect.")
            self._master = master
            for h, (_, pub) in list(self.keys.items()):
                self.keys[h] = (_core.aes256_cbc_decrypt(master, _iv(pub), self.crypted[h]), pub)
            if self.hd is not None and self.hd.get("seed_crypted"):
                iv = self.hd.get("seed_iv") or _iv(b"hdseed")
                self.hd["seed"] = _core.aes256_cbc_decrypt(master, iv, self.hd["seed_crypted"])
            if self.hd is not None and self.hd.get("ref_words_crypted"):  # imported: words, passphrase apart
                iv = self.hd["seed_iv"]
                self.hd["mnemonic"] = _core.aes256_cbc_decrypt(master, iv, self.hd["ref_words_crypted"]).decode()
                pc = self.hd.get("ref_pass_crypted")
                self.hd["mnemonic_passphrase"] = _core.aes256_cbc_decrypt(master, iv, pc).decode() if pc else ""
            if self.hd is not None and self.hd.get("mnemonic_crypted"):
                m, pp = json.loads(_core.aes256_cbc_decrypt(master, _iv(b"bip39words"), self.hd["mnemonic_crypted"]))
                self.hd["mnemonic"], self.hd["mnemonic_passphrase"] = m, pp
            if self._relock is not None:
                self._relock.cancel()
            self.unlocked_until = int(time.time()) + int(timeout) if timeout else 0
            if timeout:
                self._relock = threading.Timer(float(timeout), self.lock_wallet)
                self._relock.daemon = True
                self._relock.start()

    def lock_wallet(self) -> None:
        with self.lock:
            if self.mkey is None:
                return
            self._master = None
            for h, (_, pub) in list(self.keys.items()):
                self.keys[h] = (None, pub)
            if self.hd is not None:
                self.hd["seed"] = None
                if self.hd.get("mnemonic_crypted") or self.hd.get("ref_words_crypted"):
                    self.hd["mnemonic"] = self.hd["mnemonic_passphrase"] = None
            self.unlocked_until = 0

    def change_passphrase(self, old: str, new: str) -> None:
        with self.lock:
            if self.mkey is None:
                raise WalletError("Error: running with an unencrypted wallet, but walletpassphrasechange was called.")
            master = self._master_from(old)
            if master is None:
                raise WalletError("Error: The wallet passphrase entered was incorrect.")
            salt = os.urandom(8)
            key, iv = _core.bytes_to_key_sha512(new, salt, self.mkey["rounds"])
            self.mkey = {"salt": salt, "rounds": self.mkey["rounds"], "crypted": _core.aes256_cbc_encrypt(key, iv, master)}
            self._save()

    def _h160_of(self, address: str) -> bytes:
        raw = _core.base58check_decode(address)
        if raw is None or len(raw) != 21 or raw[0] != self.params.pubkey_prefix:
            raise WalletError("Invalid address")
        return raw[1:]

    def add_redeem_script(self, script: bytes) -> str:
        """Remember a P2SH redeem script (addmultisigaddress); returns its P2SH address."""
        h = _core.hash160(script)
        with self.lock:
            self.redeem_scripts[h] = script
            self._save()
        return _core.base58check_encode(bytes([self.params.script_prefix]) + h)

    def scripts(self) -> list[bytes]:
        """Every scriptPubKey the wallet can spend: P2PKH, P2PK, P2WPKH and P2SH-P2WPKH of each key."""
        with self.lock:
            out = []
            for h, (_, pub) in self.keys.items():
                out.append(p2pkh(h))
                out.append(_push(pub) + b"\xac")
                out.append(b"\x00\x14" + h)
            for sh in self._p2sh_wpkh:
                out.append(b"\xa9\x14" + sh + b"\x87")
            return out

    def is_mine(self, spk: bytes) -> bool:
        return self._key_for(spk) is not None

    def is_watch(self, spk: bytes) -> bool:
        """ISMINE_WATCH_ONLY: an imported script (or an asset output paying one) without a key."""
        if spk in self.watch:
            return not self.is_mine(spk)
        return len(spk) > 31 and spk[25] == 0xC0 and spk[:25] in self.watch and not self.is_mine(spk)

    def add_watch(self, spk: bytes, label: str = "", solvable: bool = False) -> None:
        """AddWatchOnly (importaddress / importpubkey / importmulti)."""
        with self.lock:
            if self.is_mine(spk):
                raise WalletError("The wallet already contains the private key for this address or script")
            self.watch[spk] = {"label": label, "solvable": solvable or self.watch.get(spk, {}).get("solvable", False)}
            self._save()

    def _key_for(self, spk: bytes):
        """(secret, pubkey, kind) for a scriptPubKey the wallet can sign, else None."""
        if len(spk) > 31 and spk[25] == 0xC0 and _core.parse_asset_script(spk) is not None:
            k = self._key_for(spk[:25])  # an asset output is spent like its P2PKH prefix
            return None if k is None or k[2] != "p2pkh" else k
        if len(spk) == 25 and spk[:3] == b"\x76\xa9\x14" and spk[23:] == b"\x88\xac":
            k = self.keys.get(spk[3:23])
            return None if k is None else (k[0], k[1], "p2pkh")
        if len(spk) == 35 and spk[0] == 33 and spk[34] == 0xac:
            h = _core.hash160(spk[1:34])
            k = self.keys.get(h)
            return None if k is None else (k[0], k[1], "p2pk")
        if len(spk) == 22 and spk[:2] == b"\x00\x14":
            k = self.keys.get(spk[2:])
            return None if k is None else (k[0], k[1], "p2wpkh")
        if len(spk) == 23 and spk[:2] == b"\xa9\x14" and spk[22] == 0x87:  # P2SH-P2WPKH of one of our keys
            h = self._p2sh_wpkh.get(spk[2:22])
            k = None if h is None else self.keys.get(h)
            return None if k is None else (k[0], k[1], "p2sh-p2wpkh")
        return None

    # ------------------------------------------------------------------ coins
    def unspent(self, minconf: int = 1, maxconf: int = 9_999_999, include_watch: bool = False) -> list[dict]:
        """AvailableCoins: wallet outputs in the UTXO set (and, for minconf 0, the pool) that the
        pool does not spend and lockunspent has not locked. Watch-only outputs (include_watch) come
        back with spendable False and watchonly True."""
        st = self.state
        with st.lock:
            tip = st.coins_tip().height
            scripts = self.scripts()
            watch = set()
            if include_watch:
                watch = {spk for spk in self.watch if spk not in set(scripts)}
                scripts = scripts + sorted(watch)
            pool_spent = {(i.prevout.hash, i.prevout.n) for e in st.mempool.values() for i in e.tx.vin}
            locked = self.history.locked if self.history is not None else set()
            out = []
            for txid, n, value, spk, height, coinbase in st.coins.outputs_for_scripts(scripts):
                conf = tip - height + 1
                if (txid, n) in pool_spent or (txid, n) in locked or not (minconf <= conf <= maxconf):
                    continue
                # CWalletTx::GetBlocksToMaturity: a coinbase needs COINBASE_MATURITY + 1 confirmations
                mature = not coinbase or conf > _core.COINBASE_MATURITY
                wo = spk in watch
                out.append({"txid": txid, "vout": n, "amount": value, "scriptPubKey": spk,
                            "confirmations": conf, "spendable": mature and not wo, "coinbase": coinbase,
                            "watchonly": wo, "mature": mature})
            if minconf <= 0:
                mine = set(scripts)
                for txid, e in st.mempool.items():
                    for n, o in enumerate(e.tx.vout):
                        if o.script_pubkey in mine and (txid, n) not in pool_spent:
                            wo = o.script_pubkey in watch
                            out.append({"txid": txid, "vout": n, "amount": o.value, "scriptPubKey": o.script_pubkey,
                                        "confirmations": 0, "spendable": not wo, "coinbase": False,
                                        "watchonly": wo, "mature": True})
            return out

    def watch_balance(self, minconf: int = 1) -> int:
        return sum(u["amount"] for u in self.unspent(minconf, include_watch=True) if u["watchonly"] and u["mature"])

    def balance(self, minconf: int = 1) -> int:
        return sum(u["amount"] for u in self.unspent(minconf) if u["spendable"])

    def immature_balance(self) -> int:
        return sum(u["amount"] for u in self.unspent(1) if not u["mature"])

    # ------------------------------------------------------------------ signing
    def sign(self, tx, prevouts: dict[tuple[bytes, int], tuple[bytes, int]], extra_keys: list[bytes] = (),
             hash_type: int = SIGHASH_ALL, redeem_scripts: dict | None = None) -> tuple[object, bool, list[dict]]:
        """SignTransaction: every input whose spent output is known and spendable by a wallet
        key (or one of `extra_keys`). Returns (tx, complete, errors)."""
        with self.lock:
            return self._sign(tx, prevouts, extra_keys, hash_type, redeem_scripts)

    def _sign_multisig(self, tx, i: int, redeem: bytes, ms: tuple, amount: int, hash_type: int) -> bool:
        """P2SH multisig input: keep the signatures already in its scriptSig, add the wallet's, in
        key order (CombineMultisig / SignStep). True once m signatures are present."""
        m, pubs = ms
        vin = tx.vin[i]
        msg = _core.signature_hash(redeem, tx.serialize(True), i, hash_type, amount, 0)
        have = {}
        for push in _pushes(vin.script_sig)[1:-1]:
            for pub in pubs:
                if pub not in have and push and _core.secp_verify(pub, push[:-1], msg):
                    have[pub] = push
                    break
        for pub in pubs:
            if pub in have or len(have) >= m:
                continue
            k = self.keys.get(_core.hash160(pub))
            if k is not None and k[1] == pub:
                have[pub] = _core.secp_sign(msg, k[0]) + bytes([hash_type])
        sigs = [have[pub] for pub in pubs if pub in have][:m]
        vin.script_sig = b"\x00" + b"".join(_push(x) for x in sigs) + _push(redeem)
        vins = list(tx.vin)
        vins[i] = vin
        tx.vin = vins
        return len(sigs) >= m

    def _sign(self, tx, prevouts, extra_keys, hash_type, redeem_scripts=None):
        redeem_scripts = redeem_scripts or {}
        extra = {}
        for sec in extra_keys:
            pub = _core.secp_pubkey_create(sec, True)
            extra[_core.hash160(pub)] = (sec, pub)
        keys = dict(self.keys)
        keys.update(extra)
        sh = dict(self._p2sh_wpkh)
        sh.update({_core.hash160(b"\x00\x14" + h): h for h in extra})
        saved, saved_sh = self.keys, self._p2sh_wpkh
        self.keys, self._p2sh_wpkh = keys, sh
        try:
            vins = list(tx.vin)
            errors = []
            for i, vin in enumerate(vins):
                prev = prevouts.get((vin.prevout.hash, vin.prevout.n))
                if prev is None:
                    errors.append({"txid": vin.prevout.hash[::-1].hex(), "vout": vin.prevout.n,
                                   "error": "Input not found or already spent"})
                    continue
                spk, amount = prev
                if len(spk) == 23 and spk[:2] == b"\xa9\x14" and spk[22] == 0x87:
                    redeem = self.redeem_scripts.get(spk[2:22]) or redeem_scripts.get(spk[2:22])
                    ms = parse_multisig(redeem) if redeem else None
                    if ms is not None:
                        tx.vin = vins
                        ok = self._sign_multisig(tx, i, redeem, ms, amount, hash_type)
                        vins = list(tx.vin)
                        if not ok:
                            errors.append({"txid": vin.prevout.hash[::-1].hex(), "vout": vin.prevout.n,
                                           "error": "Not enough signatures for the multisig input"})
                        continue
                k = self._key_for(spk)
                if k is None:
                    errors.append({"txid": vin.prevout.hash[::-1].hex(), "vout": vin.prevout.n,
                                   "error": "Unable to sign input, missing key"})
                    continue
                sec, pub, kind = k
                if sec is None:
                    raise WalletError(UNLOCK_NEEDED)
                tx.vin = vins
                raw = tx.serialize(True)
                if kind in ("p2pkh", "p2pk"):
                    msg = _core.signature_hash(spk, raw, i, hash_type, amount, 0)
                    sig = _core.secp_sign(msg, sec) + bytes([hash_type])
                    vin.script_sig = _push(sig) + (_push(pub) if kind == "p2pkh" else b"")
                    vin.witness = []
                else:
                    code = p2pkh(_core.hash160(pub))
                    msg = _core.signature_hash(code, raw, i, hash_type, amount, 1)
                    sig = _core.secp_sign(msg, sec) + bytes([hash_type])
                    vin.witness = [sig, pub]
                    vin.script_sig = _push(b"\x00\x14" + _core.hash160(pub)) if kind == "p2sh-p2wpkh" else b""
                vins[i] = vin
            tx.vin = vins
            return tx, not errors, errors
        finally:
            self.keys, self._p2sh_wpkh = saved, saved_sh

    def fund_and_sign(self, pre_outputs: list, post_outputs: list, extra_inputs: list[dict] = (),
                      fee_rate: int = DEFAULT_FEE_RATE, change_spk: bytes | None = None,
                      require_complete: bool = True):
        """A transaction whose outputs are `pre_outputs`, a CLORE change output, then `post_outputs`
        (asset transactions need their issue / reissue data last), spending `extra_inputs`
        (e.g. asset outputs: dicts with txid, vout, amount, scriptPubKey) plus CLORE coins for the
        outputs' value and the fee. Returns (tx, fee)."""
        target = sum(o.value for o in list(pre_outputs) + list(post_outputs))
        given = {(u["txid"], u["vout"]) for u in extra_inputs}
        base = sum(u["amount"] for u in extra_inputs)  # value the caller's inputs already bring
        coins = sorted((u for u in self.unspent(1) if u["spendable"] and (u["txid"], u["vout"]) not in given),
                       key=lambda u: -u["amount"])
        fee = 0
        for _ in range(20):
            need = target + fee
            chosen, total = [], base
            for u in coins:
                if total >= need:
                    break
                chosen.append(u)
                total += u["amount"]
            if total < need:
                raise WalletError("Insufficient funds")
            tx = _core.Transaction()
            tx.version = 2
            vins = []
            for u in list(extra_inputs) + chosen:
                vin = _core.TxIn()
                op = _core.OutPoint()
                op.hash, op.n = u["txid"], u["vout"]
                vin.prevout = op
                vin.sequence = 0xfffffffe
                vins.append(vin)
            tx.vin = vins
            outs = list(pre_outputs)
            change = total - need
            if change > 0:
                if change_spk is None:
                    change_spk = _core.address_to_script(self.new_address("change"), self.params.pubkey_prefix,
                                                         self.params.script_prefix)
                outs.append(_core.TxOut(change, change_spk))
            tx.vout = outs + list(post_outputs)
            tx.lock_time = max(0, self.state.coins_tip().height)
            prevs = {(u["txid"], u["vout"]): (u["scriptPubKey"], u["amount"]) for u in list(extra_inputs) + chosen}
            tx, complete, errors = self.sign(tx, prevs)
            if not complete and require_complete:
                raise WalletError(f"Signing transaction failed: {errors}")
            size = (len(tx.serialize(False)) * 3 + len(tx.serialize(True)) + 3) // 4
            size += 110 * len(errors)  # inputs left for another signer: a P2PKH-sized scriptSig each
            want = self._capped_fee(max(1, fee_rate * size // 1000))
            if fee >= want:
                return tx, fee
            fee = want + 68
        raise WalletError("Transaction fee did not converge")

    def create_transaction(self, outputs: list[tuple[bytes, int]], fee_rate: int = DEFAULT_FEE_RATE,
                           subtract_fee: bool = False, minconf: int = 1, replaceable: bool | None = None,
                           from_scripts: set | None = None, change_spk: bytes | None = None):
        """CreateTransaction: largest-first coin selection over spendable wallet outputs (only those
        paying `from_scripts` when given: sendfromaddress), a change output to a fresh key (or
        `change_spk`), fee = fee_rate per kvB of the signed size; inputs signal BIP125 when
        `replaceable` (default -walletrbf). Returns (tx, fee)."""
        if not outputs or any(v <= 0 for _, v in outputs):
            raise WalletError("Invalid amount")
        target = sum(v for _, v in outputs)
        coins = sorted((u for u in self.unspent(minconf) if u["spendable"]
                        and (from_scripts is None or u["scriptPubKey"] in from_scripts)), key=lambda u: -u["amount"])
        if minconf >= 1 and self.spend_zeroconf_change and sum(u["amount"] for u in coins) < target:
            # SelectCoins' last pass (nConfMine 0): our own unconfirmed change from trusted wallet
            # transactions, after every confirmed coin
            extra = [u for u in self.unspent(0) if u["confirmations"] == 0 and u["spendable"]
                     and (from_scripts is None or u["scriptPubKey"] in from_scripts) and self._trusted(u["txid"])]
            coins += sorted(extra, key=lambda u: -u["amount"])
        seq = 0xfffffffd if (self.walletrbf if replaceable is None else replaceable) else 0xfffffffe
        fee = 0
        for _ in range(20):  # fee depends on the size, size on the inputs chosen
            need = target + (0 if subtract_fee else fee)
            chosen, total = [], 0
            for u in coins:
                if total >= need:
                    break
                chosen.append(u)
                total += u["amount"]
            if total < need:
                raise WalletError("Insufficient funds")
            tx = _core.Transaction()
            tx.version = 2
            vins = []
            for u in chosen:
                vin = _core.TxIn()
                op = _core.OutPoint()
                op.hash, op.n = u["txid"], u["vout"]
                vin.prevout = op
                vin.sequence = seq
                vins.append(vin)
            tx.vin = vins
            outs = [_core.TxOut(v, s) for s, v in outputs]
            if subtract_fee:
                first = outs[0]
                outs[0] = _core.TxOut(first.value - fee, first.script_pubkey)
                if outs[0].value <= 0:
                    raise WalletError("The transaction amount is too small to pay the fee")
            change = total - target - (0 if subtract_fee else fee)
            if 0 < change < self._change_discard_threshold():
                # dust at the discard rate (GetDiscardRate: -discardfee, at least the dust relay fee):
                # the change goes to the fee instead of an output not worth spending
                change = 0
            if change > 0:
                if change_spk is None:
                    change_spk = _core.address_to_script(self.new_address("change"), self.params.pubkey_prefix,
                                                         self.params.script_prefix)
                outs.append(_core.TxOut(change, change_spk))
            tx.vout = outs
            tx.lock_time = max(0, self.state.coins_tip().height)  # anti fee-sniping (src/wallet/wallet.cpp)
            prevs = {(u["txid"], u["vout"]): (u["scriptPubKey"], u["amount"]) for u in chosen}
            tx, complete, errors = self.sign(tx, prevs)
            if not complete:
                raise WalletError(f"Signing transaction failed: {errors}")
            size = (len(tx.serialize(False)) * 3 + len(tx.serialize(True)) + 3) // 4
            want_fee = self._capped_fee(max(1, fee_rate * size // 1000))
            if fee >= want_fee:
                return tx, total - sum(o.value for o in outs)  # a discarded change is part of the fee
            fee = want_fee + 68  # headroom for a changed signature size
        raise WalletError("Transaction fee did not converge")

    def send(self, outputs: list[tuple[bytes, int]], subtract_fee: bool = False, comment: str = "",
             replaceable: bool | None = None, from_scripts: set | None = None, change_spk: bytes | None = None,
             comment_to: str = "", from_account: str | None = None, minconf: int = 1) -> bytes:
        """SendMoney / CommitTransaction: build, submit to the pool, record in the history."""
        tx, _ = self.create_transaction(outputs, fee_rate=self.fee_rate, subtract_fee=subtract_fee, minconf=minconf,
                                        replaceable=replaceable, from_scripts=from_scripts, change_spk=change_spk)
        if self.reject_long_chains:
            # -walletrejectlongchains: refuse what the pool's ancestor / descendant limits would refuse
            vsize = (len(tx.serialize(False)) * 3 + len(tx.serialize(True)) + 3) // 4
            with self.state.lock:
                if self.state._check_package_limits(tx, vsize, set()):
                    raise WalletError("Transaction has too long of a mempool chain")
        return self.commit(tx, comment, comment_to, from_account)

    def _change_discard_threshold(self) -> int:
        """GetDustThreshold of a P2PKH change output (34 bytes, spent by a 148-byte input) at the
        discard rate."""
        rate = max(self.discard_fee, getattr(self.state, "dust_relay_fee", 0))
        return (34 + 148) * rate // 1000

    def _trusted(self, txid: bytes) -> bool:
        """CWalletTx::IsTrusted for a pool transaction: every input spends one of our outputs."""
        e = self.state.mempool.get(txid)
        if e is None or self.history is None:
            return False
        mine = set(self.scripts())
        for i in e.tx.vin:
            prev = self.history.txs.get(i.prevout.hash)
            if prev is None or i.prevout.n >= len(prev.tx.vout) or prev.tx.vout[i.prevout.n].script_pubkey not in mine:
                return False
        return True

    def _capped_fee(self, fee: int) -> int:
        """GetMinimumFee's last step: never above -maxtxfee (CreateTransaction then reports
        "Fee exceeds maximum configured by -maxtxfee" if the cap cannot pay the relay fee)."""
        cap = self.max_tx_fee if self.max_tx_fee is not None else getattr(self.state, "max_tx_fee", None)
        if cap is not None and fee > cap:
            raise WalletError("Fee exceeds maximum configured by -maxtxfee")
        return fee

    def commit(self, tx, comment: str = "", comment_to: str = "", from_account: str | None = None) -> bytes:
        if self.broadcast:  # -walletbroadcast=0: recorded in the wallet, never submitted or relayed
            ok, reason, _ = self.state.accept_to_mempool(tx)
            if not ok:
                raise WalletError(f"Transaction rejected: {reason}")
        if self.history is not None:
            self.history.add(tx)
            w = self.history.txs.get(tx.txid())
            if w is not None and (comment or comment_to or from_account is not None):
                w.comment = comment
                w.comment_to = comment_to
                w.from_account = from_account
                self.history.save()
        return tx.txid()

    # ------------------------------------------------------------------ fee bumping (src/wallet/feebumper.cpp)
    def bump_fee(self, txid: bytes, total_fee: int | None = None, replaceable: bool = True) -> tuple[bytes, int, int]:
        """CFeeBumper: a replacement of an opted-in wallet transaction in the pool, paying the extra
        fee out of its change output. Returns (new txid, old fee, new fee)."""
        st = self.state
        with st.lock, self.lock:
            e = st.mempool.get(txid)
            if e is None:
                raise WalletError("Transaction is not in the mempool" if self.history is None or
                                  txid not in self.history.txs else "Transaction has been mined, or is conflicted "
                                  "with a mined transaction")
            tx = e.tx
            if any(i.prevout.hash == txid for x in st.mempool.values() for i in x.tx.vin):
                raise WalletError("Transaction has descendants in the wallet")
            if not any(i.sequence < 0xfffffffe for i in tx.vin):
                raise WalletError("Transaction is not BIP 125 replaceable")
            coins = []
            for i in tx.vin:
                c = st._spent_coin(i.prevout)
                if c is None or not self.is_mine(c[1]):
                    raise WalletError("Transaction contains inputs that don't belong to this wallet")
                coins.append(c)
            change = [k for k, o in enumerate(tx.vout) if self.is_mine(o.script_pubkey)
                      and self.labels.get(o.script_pubkey[3:23] if len(o.script_pubkey) == 25 else b"") == "change"]
            if len(change) != 1:
                raise WalletError("Transaction does not have a change output")
            old_fee = sum(c[0] for c in coins) - tx.value_out()
            vsize = (len(tx.serialize(False)) * 3 + len(tx.serialize(True)) + 3) // 4
            # the new signatures may come out longer (DER r and s each 32 or 33 bytes): price the
            # replacement for up to 2 more bytes per input, at a rate above the old one's actual rate,
            # so its feerate beats the original whatever lengths the new signatures get
            size = vsize + 2 * len(tx.vin)
            old_rate = -(-old_fee * 1000 // vsize)
            if total_fee is not None:
                min_total = old_rate * size // 1000 + st.incremental_relay_fee * size // 1000
                if total_fee < min_total:
                    raise WalletError(f"Insufficient totalFee, must be at least {min_total / COIN:.8f}")
                new_fee = total_fee
            else:
                rate = max(self.fee_rate, old_rate + 1 + max(WALLET_INCREMENTAL_RELAY_FEE, st.incremental_relay_fee))
                new_fee = rate * size // 1000
            k = change[0]
            ch = tx.vout[k]
            left = ch.value - (new_fee - old_fee)
            outs = list(tx.vout)
            if left < 0:
                raise WalletError("Change output is too small to bump the fee")
            if left < DUST_THRESHOLD:  # the whole change goes to the fee
                new_fee += left
                del outs[k]
            else:
                outs[k] = _core.TxOut(left, ch.script_pubkey)
            new = _core.Transaction()
            new.version, new.lock_time = tx.version, tx.lock_time
            vins = []
            for i in tx.vin:
                v = _core.TxIn()
                v.prevout = i.prevout
                v.sequence = 0xfffffffd if replaceable else 0xfffffffe
                vins.append(v)
            new.vin, new.vout = vins, outs
            prevs = {(i.prevout.hash, i.prevout.n): (c[1], c[0]) for i, c in zip(tx.vin, coins)}
            new, complete, errors = self._sign(new, prevs, (), SIGHASH_ALL)
            if not complete:
                raise WalletError(f"Can't sign transaction: {errors}")
            new_id = self.commit(new)
            if self.history is not None and txid in self.history.txs:
                self.history.txs[txid].replaced_by = new_id
                self.history.txs[new_id].replaces = txid
                self.history.save()
            return new_id, old_fee, new_fee
