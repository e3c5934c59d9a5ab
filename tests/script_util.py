"""Test helpers for the script interpreter: the reference's script assembly parser and the
crediting / spending transaction pair its script tests run in.

Parity: ParseScript (src/core_read.cpp: numbers through CScript << int64, `0x..` raw bytes,
'quoted' pushes, opcode names with or without OP_), BuildCreditingTransaction /
BuildSpendingTransaction (src/test/script_tests.cpp).
"""
from __future__ import annotations

import hashlib
import struct

# GetOpName (src/script/script.cpp) for every opcode ParseScript accepts by name: OP_RESERVED and
# everything from OP_NOP up to OP_NOP10 (OP_NOP2/3 are named CHECKLOCKTIMEVERIFY/CHECKSEQUENCEVERIFY).
OPCODES = {
    "OP_RESERVED": 0x50, "OP_NOP": 0x61, "OP_VER": 0x62, "OP_IF": 0x63, "OP_NOTIF": 0x64, "OP_VERIF": 0x65,
    "OP_VERNOTIF": 0x66, "OP_ELSE": 0x67, "OP_ENDIF": 0x68, "OP_VERIFY": 0x69, "OP_RETURN": 0x6a,
    "OP_TOALTSTACK": 0x6b, "OP_FROMALTSTACK": 0x6c, "OP_2DROP": 0x6d, "OP_2DUP": 0x6e, "OP_3DUP": 0x6f,
    "OP_2OVER": 0x70, "OP_2ROT": 0x71, "OP_2SWAP": 0x72, "OP_IFDUP": 0x73, "OP_DEPTH": 0x74, "OP_DROP": 0x75,
    "OP_DUP": 0x76, "OP_NIP": 0x77, "OP_OVER": 0x78, "OP_PICK": 0x79, "OP_ROLL": 0x7a, "OP_ROT": 0x7b,
    "OP_SWAP": 0x7c, "OP_TUCK": 0x7d, "OP_CAT": 0x7e, "OP_SUBSTR": 0x7f, "OP_LEFT": 0x80, "OP_RIGHT": 0x81,
    "OP_SIZE": 0x82, "OP_INVERT": 0x83, "OP_AND": 0x84, "OP_OR": 0x85, "OP_XOR": 0x86, "OP_EQUAL": 0x87,
    "OP_EQUALVERIFY": 0x88, "OP_RESERVED1": 0x89, "OP_RESERVED2": 0x8a, "OP_1ADD": 0x8b, "OP_1SUB": 0x8c,
    "OP_2MUL": 0x8d, "OP_2DIV": 0x8e, "OP_NEGATE": 0x8f, "OP_ABS": 0x90, "OP_NOT": 0x91, "OP_0NOTEQUAL": 0x92,
    "OP_ADD": 0x93, "OP_SUB": 0x94, "OP_MUL": 0x95, "OP_DIV": 0x96, "OP_MOD": 0x97, "OP_LSHIFT": 0x98,
    "OP_RSHIFT": 0x99, "OP_BOOLAND": 0x9a, "OP_BOOLOR": 0x9b, "OP_NUMEQUAL": 0x9c, "OP_NUMEQUALVERIFY": 0x9d,
    "OP_NUMNOTEQUAL": 0x9e, "OP_LESSTHAN": 0x9f, "OP_GREATERTHAN": 0xa0, "OP_LESSTHANOREQUAL": 0xa1,
    "OP_GREATERTHANOREQUAL": 0xa2, "OP_MIN": 0xa3, "OP_MAX": 0xa4, "OP_WITHIN": 0xa5, "OP_RIPEMD160": 0xa6,
    "OP_SHA1": 0xa7, "OP_SHA256": 0xa8, "OP_HASH160": 0xa9, "OP_HASH256": 0xaa, "OP_CODESEPARATOR": 0xab,
    "OP_CHECKSIG": 0xac, "OP_CHECKSIGVERIFY": 0xad, "OP_CHECKMULTISIG": 0xae, "OP_CHECKMULTISIGVERIFY": 0xaf,
    "OP_NOP1": 0xb0, "OP_CHECKLOCKTIMEVERIFY": 0xb1, "OP_CHECKSEQUENCEVERIFY": 0xb2, "OP_NOP4": 0xb3,
    "OP_NOP5": 0xb4, "OP_NOP6": 0xb5, "OP_NOP7": 0xb6, "OP_NOP8": 0xb7, "OP_NOP9": 0xb8, "OP_NOP10": 0xb9,
}
NAMES = dict(OPCODES)
NAMES.update({k[3:]: v for k, v in OPCODES.items()})


def scriptnum(n: int) -> bytes:
    if n == 0:
        return b""
    neg, a = n < 0, abs(n)
    out = bytearray()
    while a:
        out.append(a & 0xff)
        a >>= 8
    if out[-1] & 0x80:
        out.append(0x80 if neg else 0)
    elif neg:
        out[-1] |= 0x80
    return bytes(out)


def push_data(d: bytes) -> bytes:
    n = len(d)
    if n < 0x4c:
        return bytes([n]) + d
    if n <= 0xff:
        return b"\x4c" + bytes([n]) + d
    if n <= 0xffff:
        return b"\x4d" + struct.pack("<H", n) + d
    return b"\x4e" + struct.pack("<I", n) + d


def push_int(n: int) -> bytes:
    if n == -1 or 1 <= n <= 16:
        return bytes([n + 0x50])
    if n == 0:
        return b"\x00"
    return push_data(scriptnum(n))


def parse_script(src: str) -> bytes:
    out = bytearray()
    for w in src.replace("\t", " ").replace("\n", " ").split(" "):
        if not w:
            continue
        if w.isdigit() or (w.startswith("-") and w[1:].isdigit()):
            out += push_int(int(w))
        elif w.startswith("0x") and len(w) > 2 and all(ch in "0123456789abcdefABCDEF" for ch in w[2:]):
            out += bytes.fromhex(w[2:])
        elif len(w) >= 2 and w[0] == "'" and w[-1] == "'":
            out += push_data(w[1:-1].encode())
        elif w in NAMES:
            out.append(NAMES[w])
        else:
            raise ValueError(f"script parse error: {w!r}")
    return bytes(out)


def flags_of(s: str, bits: dict) -> int:
    f = 0
    for w in s.split(","):
        if w:
            f |= bits[w]
    return f


def _tx(version, vin, vout, locktime, witness=None) -> bytes:
    """vin: [(prev_hash32, n, script_sig, sequence)], vout: [(value, spk)]"""
    def cs(n):
        return bytes([n]) if n < 253 else b"\xfd" + struct.pack("<H", n)
    wit = witness is not None and any(witness)
    b = struct.pack("<i", version) + (b"\x00\x01" if wit else b"") + cs(len(vin))
    for h, n, ss, seq in vin:
        b += h + struct.pack("<I", n) + cs(len(ss)) + ss + struct.pack("<I", seq)
    b += cs(len(vout))
    for v, spk in vout:
        b += struct.pack("<q", v) + cs(len(spk)) + spk
    if wit:
        for stack in witness:
            b += cs(len(stack)) + b"".join(cs(len(x)) + x for x in stack)
    return b + struct.pack("<I", locktime)


def credit_spend(script_sig: bytes, script_pubkey: bytes, witness: list[bytes], amount: int) -> bytes:
    """The spending transaction of script_tests.cpp (input 0 spends the crediting tx's output 0)."""
    credit = _tx(1, [(b"\x00" * 32, 0xffffffff, b"\x00\x00", 0xffffffff)], [(amount, script_pubkey)], 0)
    txid = hashlib.sha256(hashlib.sha256(credit).digest()).digest()
    return _tx(1, [(txid, 0, script_sig, 0xffffffff)], [(amount, b"")], 0, [witness])
