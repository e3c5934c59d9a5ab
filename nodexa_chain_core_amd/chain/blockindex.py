"""Persistent block index: blocks/index.log.

Role of the reference's CBlockTreeDB (src/txdb.h:115, LevelDB `blocks/index/`): on
start-up the node rebuilds its block index from compact per-block records instead of
re-reading every block in the blk files (what `-reindex` does). LevelDB is not part
of this engine, so the store is an append-only log (one record per stored block), which
is also how the index is written: blocks are only ever added; invalidation state is
recomputed by the header chain.

Record: u32 payload length | payload | first 4 bytes of SHA256d(payload), where payload =
i32 file, u32 data offset, u32 size, u32 nTx, then the serialized block header. A torn
final record (crash mid-append) fails its checksum and is cut off on load; the blocks
written after the last good record are recovered by scanning the blk-file tail
(ThreadImport-style, chain/state.py).
"""
from __future__ import annotations

import os
import struct

from .. import core

_core = core()
_LEN = struct.Struct("<I")
_POS = struct.Struct("<iIII")


class BlockIndexLog:
    def __init__(self, path: str):
        self.path = path
        self._f = None

    def load(self) -> list[tuple[bytes, tuple[int, int, int], int]]:
        """[(header bytes, (file, offset, size), n_tx)] in append order; truncates a bad tail."""
        if not os.path.exists(self.path):
            return []
        with open(self.path, "rb") as f:
            b = f.read()
        out, off = [], 0
        while off + 4 <= len(b):
            (n,) = _LEN.unpack_from(b, off)
            end = off + 4 + n + 4
            if n < _POS.size or end > len(b):
                break
            payload = b[off + 4: off + 4 + n]
            if _core.sha256d(payload)[:4] != b[off + 4 + n: end]:
                break
            fi, fo, fs, ntx = _POS.unpack_from(payload, 0)
            out.append((payload[_POS.size:], (fi, fo, fs), ntx))
            off = end
        if off != len(b):  # torn / corrupt tail: keep the good prefix only
            with open(self.path, "r+b") as f:
                f.truncate(off)
        return out

    def append(self, header_bytes: bytes, pos, n_tx: int) -> None:
        payload = _POS.pack(pos.file, pos.offset, pos.size, n_tx) + header_bytes
        if self._f is None:
            self._f = open(self.path, "ab")
        self._f.write(_LEN.pack(len(payload)) + payload + _core.sha256d(payload)[:4])
        self._f.flush()

    def rewrite(self, records) -> None:
        """Replace the log (after a full -reindex scan): records of (header bytes, pos, n_tx)."""
        self.close()
        tmp = self.path + ".new"
        with open(tmp, "wb") as f:
            for hb, pos, ntx in records:
                payload = _POS.pack(pos.file, pos.offset, pos.size, ntx) + hb
                f.write(_LEN.pack(len(payload)) + payload + _core.sha256d(payload)[:4])
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.path)

    def sync(self) -> None:
        if self._f is not None:
            self._f.flush()
            os.fsync(self._f.fileno())

    def close(self) -> None:
        if self._f is not None:
            self.sync()
            self._f.close()
            self._f = None


def scan_blk_tail(blocks_dir: str, magic: bytes, file: int, offset: int):
    """Yield (file, data offset, raw block) for the records after byte `offset` of blk`file`
    and in every later blk file; stops at the first bad magic / short record."""
    while True:
        path = os.path.join(blocks_dir, "blk%05d.dat" % file)
        if not os.path.exists(path):
            return
        with open(path, "rb") as f:
            f.seek(offset)
            data = f.read()
        off = 0
        while off + 8 <= len(data):
            if data[off:off + 4] != magic:
                return
            (n,) = _LEN.unpack_from(data, off + 4)
            if off + 8 + n > len(data):
                return
            yield file, offset + off + 8, data[off + 8: off + 8 + n]
            off += 8 + n
        file, offset = file + 1, 0
