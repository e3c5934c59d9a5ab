"""BIP37 bloom filters and merkle blocks.

Parity (behaviour): CBloomFilter (src/bloom.h:47, src/bloom.cpp) — size / hash-function limits,
MurmurHash3 with seed n * 0xFBA4C795 + nTweak, IsRelevantAndUpdate with the BLOOM_UPDATE_*
flags; filterload / filteradd / filterclear handling and CMerkleBlock (src/merkleblock.h:130),
whose partial merkle tree is the one gettxoutproof uses (rpc/methods_ext.partial_merkle_tree).
"""
from __future__ import annotations

import math
import struct

from .. import core

_core = core()

MAX_BLOOM_FILTER_SIZE = 36000  # bytes
MAX_HASH_FUNCS = 50
MAX_SCRIPT_ELEMENT_SIZE = 520
BLOOM_UPDATE_NONE, BLOOM_UPDATE_ALL, BLOOM_UPDATE_P2PUBKEY_ONLY = 0, 1, 2
BLOOM_UPDATE_MASK = 3
LN2 = math.log(2)


def _pushes(script: bytes) -> list[bytes]:
    out, i = [], 0
    while i < len(script):
        op = script[i]
        i += 1
        n = 0
        if op < 0x4C:
            n = op
        elif op == 0x4C and i < len(script):
            n = script[i]
            i += 1
        elif op == 0x4D and i + 1 < len(script):
            n = int.from_bytes(script[i:i + 2], "little")
            i += 2
        elif op == 0x4E and i + 3 < len(script):
            n = int.from_bytes(script[i:i + 4], "little")
            i += 4
        else:
            continue
        if n:
            out.append(script[i:i + n])
        i += n
    return out


def _is_pubkey_or_multisig(spk: bytes) -> bool:
    if (len(spk) in (35, 67)) and spk[-1] == 0xAC and spk[0] in (33, 65):
        return True
    return len(spk) >= 3 and spk[-1] == 0xAE and 0x51 <= spk[0] <= 0x60


class BloomFilter:
    def __init__(self, data: bytes = b"", hash_funcs: int = 0, tweak: int = 0, flags: int = 0):
        self.data = bytearray(data)
        self.hash_funcs = hash_funcs
        self.tweak = tweak
        self.flags = flags
        self.empty = not any(self.data)
        self.full = bool(self.data) and all(b == 0xFF for b in self.data)

    @classmethod
    def create(cls, elements: int, fp_rate: float, tweak: int = 0, flags: int = BLOOM_UPDATE_ALL) -> "BloomFilter":
        size = int(min(-1 / (LN2 * LN2) * max(elements, 1) * math.log(fp_rate), MAX_BLOOM_FILTER_SIZE * 8) / 8)
        funcs = int(min(size * 8 / max(elements, 1) * LN2, MAX_HASH_FUNCS))
        return cls(bytes(max(size, 1)), max(funcs, 1), tweak, flags)

    @classmethod
    def from_payload(cls, p: bytes) -> "BloomFilter":
        n, off = _de_compact(p, 0)
        data = p[off:off + n]
        funcs, tweak, flags = struct.unpack_from("<IIB", p, off + n)
        return cls(data, funcs, tweak, flags)

    def payload(self) -> bytes:
        return _ser_compact(len(self.data)) + bytes(self.data) + struct.pack("<IIB", self.hash_funcs, self.tweak,
                                                                              self.flags)

    def within_size_constraints(self) -> bool:
        return len(self.data) <= MAX_BLOOM_FILTER_SIZE and self.hash_funcs <= MAX_HASH_FUNCS

    def _bit(self, n: int, key: bytes) -> int:
        return _core.murmur3_32((n * 0xFBA4C795 + self.tweak) & 0xFFFFFFFF, key) % (len(self.data) * 8)

    def insert(self, key: bytes) -> None:
        if self.full or not self.data:
            return
        for n in range(self.hash_funcs):
            b = self._bit(n, key)
            self.data[b >> 3] |= 1 << (b & 7)
        self.empty = False

    def contains(self, key: bytes) -> bool:
        if self.full:
            return True
        if self.empty or not self.data:
            return False
        for n in range(self.hash_funcs):
            b = self._bit(n, key)
            if not self.data[b >> 3] & (1 << (b & 7)):
                return False
        return True

    def is_relevant_and_update(self, tx) -> bool:
        """IsRelevantAndUpdate: the txid, any data push of an output (inserting the outpoint
        per the update flags), a spent outpoint we track, or a data push of a scriptSig."""
        if self.full:
            return True
        if self.empty:
            return False
        txid = tx.txid()
        found = self.contains(txid)
        for n, o in enumerate(tx.vout):
            for push in _pushes(o.script_pubkey):
                if self.contains(push):
                    found = True
                    mode = self.flags & BLOOM_UPDATE_MASK
                    if mode == BLOOM_UPDATE_ALL or (mode == BLOOM_UPDATE_P2PUBKEY_ONLY and
                                                    _is_pubkey_or_multisig(o.script_pubkey)):
                        self.insert(txid + struct.pack("<I", n))
                    break
        if found:
            return True
        for i in tx.vin:
            if self.contains(i.prevout.hash + struct.pack("<I", i.prevout.n)):
                return True
            if any(self.contains(p) for p in _pushes(i.script_sig)):
                return True
        return False


def merkle_block(block, header_bytes: bytes, filt: BloomFilter) -> tuple[bytes, list]:
    """CMerkleBlock(block, filter): header + partial merkle tree of the matched txs, and the
    matched transactions (sent after the merkleblock, as the reference does)."""
    from ..rpc.methods_ext import partial_merkle_tree

    txids, match, matched = [], [], []
    for tx in block.vtx:
        m = filt.is_relevant_and_update(tx)
        txids.append(tx.txid())
        match.append(m)
        if m:
            matched.append(tx)
    return header_bytes + partial_merkle_tree(txids, match), matched


def _ser_compact(n: int) -> bytes:
    if n < 253:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + struct.pack("<H", n)
    if n <= 0xFFFFFFFF:
        return b"\xfe" + struct.pack("<I", n)
    return b"\xff" + struct.pack("<Q", n)


def _de_compact(b: bytes, off: int) -> tuple[int, int]:
    c = b[off]
    if c < 253:
        return c, off + 1
    if c == 253:
        return struct.unpack_from("<H", b, off + 1)[0], off + 3
    if c == 254:
        return struct.unpack_from("<I", b, off + 1)[0], off + 5
    return struct.unpack_from("<Q", b, off + 1)[0], off + 9
