"""Block header (80-byte legacy / 120-byte KawPow) — bit-exact with the reference.

Parity: CBlockHeader::SerializationOp (src/primitives/block.h:59-74),
CKAWPOWInput (src/primitives/block.h:213-233), GetKAWPOWHeaderHash
(src/primitives/block.cpp:94-99), KAWPOWHash / KAWPOWHash_OnlyMix
(src/hash.cpp:258-290).

Byte-order conventions (the #1 bit-exactness hazard, SURVEY §7 "hard parts"):
  * uint256 values (prev, merkle, mix_hash, block hash) are stored as the
    reference stores them: 32 bytes, little-endian, displayed reversed (`u256_hex`).
  * KawPow consumes `header_hash = to_hash256(SHA256d(CKAWPOWInput).GetHex())`
    i.e. the SHA256d digest *byte-reversed*; `progpow_header_hash()` returns that.
  * progpow's final/mix hashes come back in storage order; the node converts
    with uint256S(to_hex(x)), i.e. it reverses them again (`from_progpow`).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

from .. import core

_core = core()


def u256_hex(b: bytes) -> str:
    """uint256::GetHex — display hex of a little-endian 32-byte value."""
    return b[::-1].hex()


def u256_from_hex(s: str) -> bytes:
    """uint256S — parse display hex into little-endian storage."""
    s = s.strip()
    if s.startswith(("0x", "0X")):
        s = s[2:]
    s = s.rjust(64, "0")[-64:]
    return bytes.fromhex(s)[::-1]


def from_progpow(h: bytes) -> bytes:
    """uint256S(to_hex(ethash_hash)) — ethash storage order -> uint256 storage."""
    return h[::-1]


def to_progpow(u: bytes) -> bytes:
    """to_hash256(uint256.GetHex()) — uint256 storage -> ethash storage order."""
    return u[::-1]


@dataclass
class BlockHeader:
    version: int = 4
    prev: bytes = bytes(32)        # uint256 storage order
    merkle_root: bytes = bytes(32)  # uint256 storage order
    time: int = 0
    bits: int = 0
    nonce: int = 0                  # legacy 32-bit nonce (X16R era)
    height: int = 0                 # KawPow fields
    nonce64: int = 0
    mix_hash: bytes = field(default=bytes(32))  # uint256 storage order

    def is_kawpow(self, kawpow_activation_time: int) -> bool:
        return self.time >= kawpow_activation_time

    def serialize(self, kawpow_activation_time: int) -> bytes:
        head = struct.pack("<i32s32sII", self.version, self.prev, self.merkle_root, self.time, self.bits)
        if not self.is_kawpow(kawpow_activation_time):
            return head + struct.pack("<I", self.nonce)
        return head + struct.pack("<IQ32s", self.height, self.nonce64, self.mix_hash)

    @classmethod
    def deserialize(cls, data: bytes, kawpow_activation_time: int, offset: int = 0) -> tuple["BlockHeader", int]:
        version, prev, merkle, t, bits = struct.unpack_from("<i32s32sII", data, offset)
        off = offset + 76
        h = cls(version, prev, merkle, t, bits)
        if t < kawpow_activation_time:
            (h.nonce,) = struct.unpack_from("<I", data, off)
            off += 4
        else:
            h.height, h.nonce64, h.mix_hash = struct.unpack_from("<IQ32s", data, off)
            off += 44
        return h, off

    def kawpow_input(self) -> bytes:
        """80-byte CKAWPOWInput preimage (no nonce64 / mix_hash)."""
        return struct.pack("<i32s32sIII", self.version, self.prev, self.merkle_root, self.time, self.bits,
                           self.height)

    def kawpow_header_hash(self) -> bytes:
        """GetKAWPOWHeaderHash(): SHA256d of CKAWPOWInput, uint256 storage order."""
        return _core.sha256d(self.kawpow_input())

    def progpow_header_hash(self) -> bytes:
        """The 32 bytes progpow::hash receives (byte-reversed SHA256d)."""
        return to_progpow(self.kawpow_header_hash())

    def legacy_bytes(self) -> bytes:
        """The 80 bytes X16R/X16RV2 hash (nVersion .. nNonce)."""
        return struct.pack("<i32s32sIII", self.version, self.prev, self.merkle_root, self.time, self.bits,
                           self.nonce)

    def hash_mix_only(self) -> bytes:
        """KAWPOWHash_OnlyMix — block hash trusting mix_hash (uint256 storage)."""
        fin = _core.kawpow_hash_no_verify(self.height, self.progpow_header_hash(), to_progpow(self.mix_hash),
                                          self.nonce64)
        return from_progpow(fin)

    def hash_full(self, ctx=None) -> tuple[bytes, bytes]:
        """KAWPOWHash — (block hash, computed mix_hash), both uint256 storage, light mode."""
        if ctx is None:
            ctx = _core.get_epoch_context(self.height // _core.EPOCH_LENGTH)
        fin, mix = _core.kawpow_hash(ctx, self.height, self.progpow_header_hash(), self.nonce64)
        return from_progpow(fin), from_progpow(mix)


def compact_to_target(bits: int) -> tuple[int, bool, bool]:
    """arith_uint256::SetCompact -> (target, negative, overflow) (src/arith_uint256.cpp:209-227)."""
    size = bits >> 24
    word = bits & 0x007FFFFF
    if size <= 3:
        word >>= 8 * (3 - size)
        target = word
    else:
        target = word << (8 * (size - 3))
    negative = word != 0 and (bits & 0x00800000) != 0
    overflow = word != 0 and ((size > 34) or (word > 0xFF and size > 33) or (word > 0xFFFF and size > 32))
    return target & ((1 << 256) - 1), negative, overflow


def target_to_compact(target: int) -> int:
    """arith_uint256::GetCompact (src/arith_uint256.cpp:229-248)."""
    size = (target.bit_length() + 7) // 8
    if size <= 3:
        compact = (target << (8 * (3 - size))) & 0xFFFFFFFF
    else:
        compact = (target >> (8 * (size - 3))) & 0xFFFFFFFF
    if compact & 0x00800000:
        compact >>= 8
        size += 1
    return (compact | (size << 24)) & 0xFFFFFFFF


def target_bytes_progpow(target: int) -> bytes:
    """A 256-bit target as an ethash boundary (big-endian bytes)."""
    return target.to_bytes(32, "big")
