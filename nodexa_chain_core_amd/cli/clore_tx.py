"""clore-tx: offline transaction creation and mutation.

Parity (behaviour): src/clore-tx.cpp — `-create`, `-json`, `-txid`, a hex transaction (or `-` for
stdin) followed by commands applied in order: nversion=N, locktime=N, replaceable(=N), in=TXID:VOUT(:SEQ),
delin=N, delout=N, outaddr=VALUE:ADDRESS, outpubkey=VALUE:PUBKEY[:FLAGS], outmultisig=VALUE:REQUIRED:PUBKEYS:
PUBKEY1:...[:FLAGS], outscript=VALUE:SCRIPT[:FLAGS], outdata=[VALUE:]DATA, sign=SIGHASH-FLAGS, load=NAME:FILE,
set=NAME:JSON (registers `prevtxs` and `privatekeys` feed `sign`). FLAGS: W wraps in P2WSH / P2WPKH, S in
P2SH. JSON output follows TxToUniv (ScriptToAsmStr with signature-hash decoding in scriptSigs).

Address version bytes come from -main (default) / -testnet / -regtest; -pubkeyprefix / -scriptprefix /
-secretprefix override them (the reference's util test vectors were generated with Bitcoin's 0 / 5 / 128).
"""
from __future__ import annotations

import hashlib
import json
import sys

from .. import core
from ..rpc.methods_ext import _OPS, _scriptnum_value, script_type

_core = core()
COIN = 100_000_000
SIGHASH = {"ALL": 1, "NONE": 2, "SINGLE": 3, "ALL|ANYONECANPAY": 0x81, "NONE|ANYONECANPAY": 0x82,
           "SINGLE|ANYONECANPAY": 0x83}
SIGHASH_NAMES = {v: k for k, v in SIGHASH.items()}
_NAME_TO_OP = {v: k for k, v in _OPS.items() if v.startswith("OP_")}
_NAME_TO_OP.update({"OP_FALSE": 0x00, "OP_TRUE": 0x51, "OP_0": 0x00, "OP_1NEGATE": 0x4F})
_NAME_TO_OP.update({f"OP_{n}": 0x50 + n for n in range(1, 17)})


class TxError(Exception):
    pass


class Ctx:
    def __init__(self, pubkey_prefix: int, script_prefix: int, secret_prefix: int):
        self.pk, self.sh, self.sec = pubkey_prefix, script_prefix, secret_prefix
        self.registers: dict[str, object] = {}

    def address(self, spk: bytes):
        return _core.script_to_address(spk, self.pk, self.sh) or None

    def spk_of(self, address: str) -> bytes:
        spk = _core.address_to_script(address, self.pk, self.sh)
        if spk is None:
            raise TxError("invalid TX output address")
        return spk


def _push(d: bytes) -> bytes:
    return _core.script_push_data(d)


def _amount(s: str) -> int:
    try:
        v = round(float(s) * COIN)
    except ValueError:
        raise TxError("invalid TX output value")
    if v < 0 or v > 1_300_000_000 * COIN:
        raise TxError("invalid TX output value")
    return v


def _hash160(b: bytes) -> bytes:
    return _core.hash160(b)


def _wrap(spk: bytes, flags: str, ctx: Ctx) -> bytes:
    if "W" in flags:
        spk = b"\x00\x20" + hashlib.sha256(spk).digest()
    if "S" in flags:
        spk = b"\xa9\x14" + _hash160(spk) + b"\x87"
    return spk


def parse_script(s: str) -> bytes:
    """ParseScript (src/core_read.cpp): numbers, 0x raw bytes, 'quoted strings', opcode names."""
    out = b""
    for w in s.split():
        if not w:
            continue
        if w.lstrip("-").isdigit():
            out += _core.script_push_int(int(w))
        elif w.startswith("0x") and len(w) > 2:
            out += bytes.fromhex(w[2:])
        elif len(w) >= 2 and w[0] == "'" and w[-1] == "'":
            out += _push(w[1:-1].encode())
        elif w in _NAME_TO_OP or ("OP_" + w) in _NAME_TO_OP:
            op = _NAME_TO_OP.get(w, _NAME_TO_OP.get("OP_" + w))
            if op is None or (0x01 <= op <= 0x4E):
                raise TxError("script parse error")
            out += bytes([op])
        else:
            raise TxError("script parse error")
    return out


# ------------------------------------------------------------------ JSON (TxToUniv)
def _strict_der(sig: bytes) -> bool:
    """IsValidSignatureEncoding (BIP66) over the signature with its hash-type byte."""
    if len(sig) < 9 or len(sig) > 73 or sig[0] != 0x30 or sig[1] != len(sig) - 3:
        return False
    rlen = sig[3]
    if 5 + rlen >= len(sig):
        return False
    slen = sig[5 + rlen]
    if rlen + slen + 7 != len(sig) or sig[2] != 0x02 or rlen == 0 or sig[4] & 0x80:
        return False
    if rlen > 1 and sig[4] == 0 and not sig[5] & 0x80:
        return False
    if sig[rlen + 4] != 0x02 or slen == 0 or sig[rlen + 6] & 0x80:
        return False
    return not (slen > 1 and sig[rlen + 6] == 0 and not sig[rlen + 7] & 0x80)


def script_asm(spk: bytes, sighash_decode: bool = False) -> str:
    out, i = [], 0
    while i < len(spk):
        op = spk[i]
        i += 1
        if 0x01 <= op <= 0x4E:
            if op < 0x4C:
                n = op
            else:
                w = {0x4C: 1, 0x4D: 2, 0x4E: 4}[op]
                if i + w > len(spk):
                    out.append("[error]")
                    break
                n = int.from_bytes(spk[i:i + w], "little")
                i += w
            if i + n > len(spk):
                out.append("[error]")
                break
            data = spk[i:i + n]
            i += n
            if n <= 4:
                out.append(str(_scriptnum_value(data)))
            elif sighash_decode and _strict_der(data) and data[-1] in SIGHASH_NAMES:
                out.append(data[:-1].hex() + "[" + SIGHASH_NAMES[data[-1]] + "]")
            else:
                out.append(data.hex())
        else:
            out.append(_OPS.get(op, "OP_UNKNOWN"))
    return " ".join(out)


def _spk_json(spk: bytes, ctx: Ctx) -> dict:
    typ = script_type(spk)
    out = {"asm": script_asm(spk), "hex": spk.hex()}
    addrs, req = [], 0
    if typ in ("pubkeyhash", "scripthash"):
        addrs, req = [ctx.address(spk)], 1
    elif typ == "pubkey":
        addrs, req = [ctx.address(b"\x76\xa9\x14" + _hash160(spk[1:-1]) + b"\x88\xac")], 1
    elif typ == "multisig":
        from ..wallet.wallet import parse_multisig

        ms = parse_multisig(spk)
        if ms is not None:
            req = ms[0]
            addrs = [ctx.address(b"\x76\xa9\x14" + _hash160(p) + b"\x88\xac") for p in ms[1]]
    if addrs and all(addrs):
        out["reqSigs"] = req
    out["type"] = typ
    if addrs and all(addrs):
        out["addresses"] = addrs
    return out


def tx_json(tx, ctx: Ctx) -> dict:
    vin = []
    for i in tx.vin:
        if i.prevout.is_null():
            e = {"coinbase": i.script_sig.hex()}
        else:
            e = {"txid": i.prevout.hash[::-1].hex(), "vout": i.prevout.n,
                 "scriptSig": {"asm": script_asm(i.script_sig, True), "hex": i.script_sig.hex()}}
        if i.witness:
            e["txinwitness"] = [w.hex() for w in i.witness]
        e["sequence"] = i.sequence
        vin.append(e)
    vout = [{"value": o.value / COIN, "n": n, "scriptPubKey": _spk_json(o.script_pubkey, ctx)}
            for n, o in enumerate(tx.vout)]
    raw = tx.serialize(True)
    return {"txid": tx.txid()[::-1].hex(), "hash": tx.wtxid()[::-1].hex(), "version": tx.version, "size": len(raw),
            "vsize": (len(tx.serialize(False)) * 3 + len(raw) + 3) // 4, "locktime": tx.lock_time, "vin": vin,
            "vout": vout, "hex": raw.hex()}


# ------------------------------------------------------------------ mutations
def _out(tx, value: int, spk: bytes) -> None:
    tx.vout = list(tx.vout) + [_core.TxOut(value, spk)]


def _pubkey(h: str) -> bytes:
    try:
        raw = bytes.fromhex(h)
    except ValueError:
        raise TxError("invalid TX output pubkey")
    if _core.secp_pubkey_normalize(raw, len(raw) == 33) is None:
        raise TxError("invalid TX output pubkey")
    return raw


def apply(tx, cmd: str, arg: str, ctx: Ctx) -> None:
    if cmd == "nversion":
        v = int(arg)
        if v < 1 or v > 2:
            raise TxError("Invalid TX version requested")
        tx.version = v
    elif cmd == "locktime":
        v = int(arg)
        if v < 0 or v > 0xFFFFFFFF:
            raise TxError("Invalid TX locktime requested")
        tx.lock_time = v
    elif cmd == "replaceable":
        vins = list(tx.vin)
        idx = int(arg) if arg else -1
        if idx >= len(vins):
            raise TxError("Invalid TX input index")
        for k, v in enumerate(vins):
            if (idx < 0 or k == idx) and v.sequence > 0xFFFFFFFD:
                v.sequence = 0xFFFFFFFD
                vins[k] = v
        tx.vin = vins
    elif cmd == "in":
        parts = arg.split(":")
        if len(parts) not in (2, 3) or len(parts[0]) != 64:
            raise TxError("TX input missing separator" if len(parts) < 2 else "invalid TX input txid")
        try:
            h = bytes.fromhex(parts[0])[::-1]
            n = int(parts[1])
        except ValueError:
            raise TxError("invalid TX input vout")
        vin = _core.TxIn()
        op = _core.OutPoint()
        op.hash, op.n = h, n
        vin.prevout = op
        vin.sequence = int(parts[2]) if len(parts) == 3 else 0xFFFFFFFF
        tx.vin = list(tx.vin) + [vin]
    elif cmd == "delin":
        k = int(arg)
        if k < 0 or k >= len(tx.vin):
            raise TxError(f"Invalid TX input index '{arg}'")
        vins = list(tx.vin)
        del vins[k]
        tx.vin = vins
    elif cmd == "delout":
        k = int(arg)
        if k < 0 or k >= len(tx.vout):
            raise TxError(f"Invalid TX output index '{arg}'")
        vouts = list(tx.vout)
        del vouts[k]
        tx.vout = vouts
    elif cmd == "outaddr":
        parts = arg.split(":")
        if len(parts) != 2:
            raise TxError("TX output missing or too many separators")
        _out(tx, _amount(parts[0]), ctx.spk_of(parts[1]))
    elif cmd == "outpubkey":
        parts = arg.split(":")
        if len(parts) < 2 or len(parts) > 3:
            raise TxError("TX output missing or too many separators")
        flags = parts[2].upper() if len(parts) == 3 else ""
        if flags and set(flags) - set("WS"):
            raise TxError("invalid TX output flags")
        pub = _pubkey(parts[1])
        if "W" in flags:
            if len(pub) != 33:
                raise TxError("Uncompressed pubkeys are not useable for SegWit outputs")
            spk = b"\x00\x14" + _hash160(pub)
            if "S" in flags:
                spk = b"\xa9\x14" + _hash160(spk) + b"\x87"
        else:
            spk = _push(pub) + b"\xac"
            if "S" in flags:
                spk = b"\xa9\x14" + _hash160(spk) + b"\x87"
        _out(tx, _amount(parts[0]), spk)
    elif cmd == "outmultisig":
        parts = arg.split(":")
        if len(parts) < 3:
            raise TxError("Not enough multisig parameters")
        value, req, n = _amount(parts[0]), int(parts[1]), int(parts[2])
        keys = parts[3:3 + n]
        rest = parts[3 + n:]
        if len(keys) != n or len(rest) > 1 or n < 1 or n > 16 or req < 1 or req > n:
            raise TxError("multisig value greater than number of keys" if req > n else "incorrect number of multisig pubkeys")
        flags = rest[0].upper() if rest else ""
        pubs = [_pubkey(k) for k in keys]
        from ..wallet.wallet import multisig_script

        script = multisig_script(req, pubs)
        if "W" in flags:
            if any(len(p) != 33 for p in pubs):
                raise TxError("Uncompressed pubkeys are not useable for SegWit outputs")
            script = b"\x00\x20" + hashlib.sha256(script).digest()
        if "S" in flags:
            if len(script) > 520:
                raise TxError("redeemScript exceeds size limit")
            script = b"\xa9\x14" + _hash160(script) + b"\x87"
        _out(tx, value, script)
    elif cmd == "outdata":
        value, data = 0, arg
        if ":" in arg:
            v, _, data = arg.partition(":")
            value = _amount(v)
        try:
            raw = bytes.fromhex(data)
        except ValueError:
            raise TxError("invalid TX output data")
        _out(tx, value, b"\x6a" + _push(raw))
    elif cmd == "outscript":
        parts = arg.split(":")
        if len(parts) < 2 or len(parts) > 3:
            raise TxError("TX output missing or too many separators")
        flags = parts[2].upper() if len(parts) == 3 else ""
        script = parse_script(parts[1])
        _out(tx, _amount(parts[0]), _wrap(script, flags, ctx))
    elif cmd == "sign":
        _sign(tx, arg, ctx)
    elif cmd in ("load", "set"):
        name, _, val = arg.partition(":")
        if not name or not val:
            raise TxError(f"{cmd} command requires NAME:{'FILENAME' if cmd == 'load' else 'JSON-STRING'}")
        text = open(val).read() if cmd == "load" else val
        try:
            ctx.registers[name] = json.loads(text)
        except ValueError:
            raise TxError(f"Cannot parse JSON for key {name}")
    else:
        raise TxError(f"unknown command: {cmd}")


def _sign(tx, flags: str, ctx: Ctx) -> None:
    ht = SIGHASH.get(flags or "ALL")
    if ht is None:
        raise TxError("unknown sighash flag/sign option")
    keys = {}
    for wif in ctx.registers.get("privatekeys", []) or []:
        raw = _core.base58check_decode(str(wif))
        if raw is None or raw[0] != ctx.sec or len(raw) not in (33, 34):
            raise TxError("privatekey not valid")
        compressed = len(raw) == 34
        pub = _core.secp_pubkey_create(raw[1:33], compressed)
        keys[_hash160(pub)] = (raw[1:33], pub)
    prev = {}
    for d in ctx.registers.get("prevtxs", []) or []:
        try:
            h = bytes.fromhex(d["txid"])[::-1]
            prev[(h, int(d["vout"]))] = (bytes.fromhex(d["scriptPubKey"]), round(float(d.get("amount", 0)) * COIN),
                                         bytes.fromhex(d["redeemScript"]) if d.get("redeemScript") else None)
        except (KeyError, ValueError, TypeError):
            raise TxError("prevtxs internal object typecheck fail")
    vins = list(tx.vin)
    for i, vin in enumerate(vins):
        p = prev.get((vin.prevout.hash, vin.prevout.n))
        if p is None:
            continue
        spk, amount, redeem = p
        if ht & 0x1F == 3 and i >= len(tx.vout):
            continue  # SIGHASH_SINGLE without a matching output is not signed
        tx.vin = vins
        raw = tx.serialize(True)
        if len(spk) == 25 and spk[:3] == b"\x76\xa9\x14":
            k = keys.get(spk[3:23])
            if k:
                sig = _core.secp_sign(_core.signature_hash(spk, raw, i, ht, amount, 0), k[0]) + bytes([ht])
                vin.script_sig = _push(sig) + _push(k[1])
        elif len(spk) in (35, 67) and spk[-1] == 0xAC:
            k = keys.get(_hash160(spk[1:-1]))
            if k:
                vin.script_sig = _push(_core.secp_sign(_core.signature_hash(spk, raw, i, ht, amount, 0), k[0]) + bytes([ht]))
        elif len(spk) == 22 and spk[:2] == b"\x00\x14":
            k = keys.get(spk[2:])
            if k:
                code = b"\x76\xa9\x14" + spk[2:] + b"\x88\xac"
                vin.witness = [_core.secp_sign(_core.signature_hash(code, raw, i, ht, amount, 1), k[0]) + bytes([ht]), k[1]]
        elif len(spk) == 23 and spk[:2] == b"\xa9\x14" and redeem:
            from ..wallet.wallet import parse_multisig

            ms = parse_multisig(redeem)
            if ms:
                msg = _core.signature_hash(redeem, raw, i, ht, amount, 0)
                sigs = [_core.secp_sign(msg, keys[_hash160(pk)][0]) + bytes([ht]) for pk in ms[1] if _hash160(pk) in keys]
                vin.script_sig = b"\x00" + b"".join(_push(s) for s in sigs[:ms[0]]) + _push(redeem)
        vins[i] = vin
    tx.vin = vins


def main(argv: list[str] | None = None, stdin=None, stdout=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    stdout = stdout or sys.stdout
    opts = {}
    while argv and argv[0].startswith("-") and argv[0] != "-":
        k, _, v = argv.pop(0).lstrip("-").partition("=")
        opts[k] = v
    net = "regtest" if "regtest" in opts else "test" if "testnet" in opts else "main"
    params = _core.make_chain_params(net)
    secret = {"main": 112, "test": 114, "regtest": 114}[net]
    ctx = Ctx(int(opts.get("pubkeyprefix", params.pubkey_prefix)), int(opts.get("scriptprefix", params.script_prefix)),
              int(opts.get("secretprefix", secret)))
    try:
        if "create" in opts:
            tx = _core.Transaction()
            tx.version = 2
        else:
            if not argv:
                raise TxError("too few parameters")
            src = argv.pop(0)
            if src == "-":
                src = (stdin or sys.stdin).read().strip()
            tx = None
            for witness in (False, True):  # DecodeHexTx(fTryNoWitness): a complete non-witness parse wins
                try:
                    tx = _core.Transaction.deserialize(bytes.fromhex(src), witness)
                    break
                except Exception:  # noqa: BLE001
                    continue
            if tx is None:
                raise TxError("invalid transaction encoding")
        for a in argv:
            cmd, _, arg = a.partition("=")
            apply(tx, cmd, arg, ctx)
    except (TxError, ValueError) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    if "txid" in opts:
        print(tx.txid()[::-1].hex(), file=stdout)
    elif "json" in opts:
        print(json.dumps(tx_json(tx, ctx), indent=4), file=stdout)
    else:
        print(tx.serialize(True).hex(), file=stdout)
    return 0


if __name__ == "__main__":
    sys.exit(main())
