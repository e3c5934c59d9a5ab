"""BIP152 compact blocks.

Parity (behaviour): CBlockHeaderAndShortTxIDs / PartiallyDownloadedBlock / BlockTransactions
(src/blockencodings.h:135-210, src/blockencodings.cpp) and the sendcmpct / cmpctblock /
getblocktxn / blocktxn handling of src/net_processing.cpp. Short ids are the low 48 bits of
SipHash-2-4 of the wtxid (version 2) or txid (version 1), keyed by the first 16 bytes of
SHA256(header || nonce); the coinbase is always prefilled; differential indexes as in the BIP.
"""
from __future__ import annotations

import hashlib
import os
import struct

from .. import core
from .bloom import _de_compact, _ser_compact

_core = core()
SHORTID_MASK = (1 << 48) - 1
# More transactions than fit a maximum-size block (8 MB / 60-byte minimum tx) is malformed.
MAX_COMPACT_TXS = 1_000_000


def _keys(header_bytes: bytes, nonce: int) -> tuple[int, int]:
    h = hashlib.sha256(header_bytes + struct.pack("<Q", nonce)).digest()
    return int.from_bytes(h[0:8], "little"), int.from_bytes(h[8:16], "little")


def short_id(k0: int, k1: int, txhash: bytes) -> int:
    return _core.siphash_uint256(k0, k1, txhash) & SHORTID_MASK


class CompactBlock:
    def __init__(self, header, header_bytes: bytes, nonce: int, shortids: list[int], prefilled: list[tuple[int, object]]):
        self.header, self.header_bytes, self.nonce = header, header_bytes, nonce
        self.shortids, self.prefilled = shortids, prefilled

    @classmethod
    def from_block(cls, block, act: int, version: int = 2, nonce: int | None = None) -> "CompactBlock":
        nonce = int.from_bytes(os.urandom(8), "little") if nonce is None else nonce
        hb = block.header.serialize(act)
        k0, k1 = _keys(hb, nonce)
        ids = [short_id(k0, k1, tx.wtxid() if version == 2 else tx.txid()) for tx in block.vtx[1:]]
        return cls(block.header, hb, nonce, ids, [(0, block.vtx[0])])

    def payload(self, witness: bool = True) -> bytes:
        out = self.header_bytes + struct.pack("<Q", self.nonce) + _ser_compact(len(self.shortids))
        out += b"".join(struct.pack("<Q", s)[:6] for s in self.shortids)
        out += _ser_compact(len(self.prefilled))
        last = -1
        for idx, tx in self.prefilled:
            out += _ser_compact(idx - last - 1) + tx.serialize(witness)
            last = idx
        return out

    @classmethod
    def from_payload(cls, p: bytes, act: int) -> "CompactBlock":
        header, off = _core.BlockHeader.deserialize_prefix(p, act, 0)
        hb = p[:off]
        (nonce,) = struct.unpack_from("<Q", p, off)
        off += 8
        n, off = _de_compact(p, off)
        # the declared count is peer-controlled (CompactSize up to 2^64): bound it by the bytes
        # actually present and by the block-size cap before building anything
        if n > MAX_COMPACT_TXS or n > (len(p) - off) // 6:
            raise ValueError("cmpctblock short-id count exceeds the payload")
        ids = [int.from_bytes(p[off + 6 * i:off + 6 * i + 6], "little") for i in range(n)]
        off += 6 * n
        m, off = _de_compact(p, off)
        if n + m > MAX_COMPACT_TXS or m > len(p) - off:
            raise ValueError("cmpctblock prefilled count exceeds the payload")
        prefilled, last = [], -1
        for _ in range(m):
            d, off = _de_compact(p, off)
            tx, used = _core.Transaction.deserialize_prefix(p, off)
            off += used
            last += d + 1
            prefilled.append((last, tx))
        return cls(header, hb, nonce, ids, prefilled)

    def reconstruct(self, pool_txs, version: int = 2):
        """PartiallyDownloadedBlock::InitData: fill from prefilled + pool transactions.
        Returns (slots, missing indexes); a short-id collision in the pool leaves the slot empty."""
        total = len(self.shortids) + len(self.prefilled)
        slots: list = [None] * total
        for idx, tx in self.prefilled:
            if idx >= total:
                raise ValueError("prefilled index out of range")
            slots[idx] = tx
        k0, k1 = _keys(self.header_bytes, self.nonce)
        want: dict[int, int] = {}
        free = [i for i in range(total) if slots[i] is None]
        for pos, sid in zip(free, self.shortids):
            if sid in want:  # duplicate short id inside the block: request both
                want[sid] = -1
            else:
                want[sid] = pos
        seen: dict[int, int] = {}
        for tx in pool_txs:
            sid = short_id(k0, k1, tx.wtxid() if version == 2 else tx.txid())
            pos = want.get(sid)
            if pos is None or pos < 0:
                continue
            seen[sid] = seen.get(sid, 0) + 1
            slots[pos] = tx if seen[sid] == 1 else None  # two pool txs with one short id: ask the peer
        missing = [i for i in range(total) if slots[i] is None]
        return slots, missing


def getblocktxn_payload(block_hash: bytes, indexes: list[int]) -> bytes:
    out, last = block_hash + _ser_compact(len(indexes)), -1
    for i in indexes:
        out += _ser_compact(i - last - 1)
        last = i
    return out


def parse_getblocktxn(p: bytes) -> tuple[bytes, list[int]]:
    h = p[:32]
    n, off = _de_compact(p, 32)
    if n > len(p) - off:  # every index takes at least one byte
        raise ValueError("getblocktxn index count exceeds the payload")
    out, last = [], -1
    for _ in range(n):
        d, off = _de_compact(p, off)
        last += d + 1
        if last > 0xFFFF:  # BlockTransactionsRequest: differential index overflowed 16 bits
            raise ValueError("getblocktxn index out of range")
        out.append(last)
    return h, out


def blocktxn_payload(block_hash: bytes, txs: list, witness: bool = True) -> bytes:
    return block_hash + _ser_compact(len(txs)) + b"".join(t.serialize(witness) for t in txs)


def parse_blocktxn(p: bytes) -> tuple[bytes, list]:
    h = p[:32]
    n, off = _de_compact(p, 32)
    if n > len(p) - off:
        raise ValueError("blocktxn count exceeds the payload")
    txs = []
    for _ in range(n):
        tx, used = _core.Transaction.deserialize_prefix(p, off)
        off += used
        txs.append(tx)
    return h, txs
