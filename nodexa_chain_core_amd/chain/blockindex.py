"""Persistent block index: blocks/index/ (BlockTreeDB, the default) or blocks/index.log.

Role of the reference's CBlockTreeDB (src/txdb.h:115, LevelDB `blocks/index/`): on
start-up the node rebuilds its block index from compact per-block records instead of
re-reading every block in the blk files (what `-reindex` does). `BlockTreeDB` keeps those
records in the reference's own LevelDB layout (csrc/store/ldb.cpp + chaindb.cpp), so the
two implementations can open each other's datadirs. `BlockIndexLog` is the earlier
append-only log of this engine (one record per stored block), kept for datadirs that use
it (-dbformat=journal).

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

    def append(self, header_bytes: bytes, pos, n_tx: int, **_) -> None:
        payload = _POS.pack(pos.file, pos.offset, pos.size, n_tx) + header_bytes
        if self._f is None:
            self._f = open(self.path, "ab")
        self._f.write(_LEN.pack(len(payload)) + payload + _core.sha256d(payload)[:4])
        self._f.flush()

    def prune_file(self, fi: int) -> list[bytes]:
        """PruneOneBlockFile (src/validation.cpp:12208-12240): every block stored in blk`fi` loses
        its data and undo (status bits and positions cleared, the header stays), and the file's
        CBlockFileInfo is reset. Returns the blocks' hashes."""
        hit = [h for h, e in self.entries.items() if e[3] == fi and e[1] & (BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)]
        for h in hit:
            e = self.entries[h]
            e[1] &= ~(BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)
            e[3] = e[4] = e[5] = 0
        self.files[fi] = [0, 0, 0, 0, 0, 0, 0]
        self.db.write([self._index_op(h) for h in hit] + [self._file_op(fi)])
        return hit

    def rewrite(self, records) -> None:
        """Replace the log (after a full -reindex scan): records of (header bytes, pos, n_tx, ...)."""
        self.close()
        tmp = self.path + ".new"
        with open(tmp, "wb") as f:
            for hb, pos, ntx, *_ in records:
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


BLOCK_VALID_TRANSACTIONS, BLOCK_VALID_SCRIPTS, BLOCK_VALID_MASK = 3, 5, 7
BLOCK_HAVE_DATA, BLOCK_HAVE_UNDO = 8, 16
BLOCK_FAILED_VALID, BLOCK_FAILED_CHILD = 32, 64
_I32 = struct.Struct("<i")


class BlockTreeDB:
    """blocks/index/ in the reference's LevelDB layout (CBlockTreeDB, src/txdb.cpp:23-38, 180-260).

    One 'b' record (CDiskBlockIndex: height, status, nTx, file / data / undo positions, header)
    per stored block, 'f' + i32 CBlockFileInfo per blk file, 'l' the last blk file, 'R' while a
    reindex runs, 'F' + name for flags; values XOR-ed with the store's obfuscation key. A datadir
    written by the reference loads from these records without -reindex, and one written here
    opens in the reference. Records are written unsynced as blocks arrive (they sit in the store's
    write-ahead log) and made durable by `sync()` at each chain-state flush, as the reference's
    FlushStateToDisk does with WriteBatchSync.
    """

    def __init__(self, path: str, kawpow_activation_time: int):
        self.path = path
        self.act = kawpow_activation_time
        self.db = _core.LevelDB(path, write_buffer_size=8 << 20)
        self.obf = _core.chaindb_obfuscation_key(self.db, True)
        self.files: dict[int, list[int]] = {}  # blocks, size, undo size, height first/last, time first/last
        self.entries: dict[bytes, list] = {}    # hash -> [height, status, ntx, file, data_pos, undo_pos, header]
        for k, v in self.db.items(b"f", b"g"):
            if len(k) == 5:
                fi = _core.decode_file_info(self._x(v))
                if fi is not None:
                    self.files[_I32.unpack(k[1:])[0]] = list(fi)
        v = self.db.get(b"l")
        self.last_file = _I32.unpack(self._x(v))[0] if v is not None and len(v) == 4 else 0

    def _x(self, v: bytes) -> bytes:
        return _core.chaindb_xor(v, self.obf)

    def load(self) -> list[tuple]:
        """Every 'b' record as (hash, height, status, ntx, file, data_pos, undo_pos, header bytes),
        in height order (parents first)."""
        recs, bad = _core.load_block_index_ldb(self.db, self.obf, self.act)
        if bad:
            raise IOError(f"{bad} unreadable block index record(s) in {self.path}")
        recs.sort(key=lambda r: r[1])
        for h, height, status, ntx, fi, dpos, upos, hb in recs:
            self.entries[h] = [height, status, ntx, fi, dpos, upos, hb]
        return recs

    def _index_op(self, h: bytes) -> tuple[bytes, bytes]:
        height, status, ntx, fi, dpos, upos, hb = self.entries[h]
        return b"b" + h, self._x(_core.encode_disk_index(height, status, ntx, fi, dpos, upos, hb, self.act))

    def _file_op(self, fi: int) -> tuple[bytes, bytes]:
        return b"f" + _I32.pack(fi), self._x(_core.encode_file_info(*self.files[fi]))

    def append(self, header_bytes: bytes, pos, n_tx: int, height: int = 0, block_hash: bytes = b"",
               time: int = 0) -> None:
        """A block's data was stored at `pos` (BLOCK_HAVE_DATA, transactions valid)."""
        old = self.entries.get(block_hash)
        status = BLOCK_HAVE_DATA | max(BLOCK_VALID_TRANSACTIONS, old[1] & BLOCK_VALID_MASK if old else 0)
        upos = 0
        if old is not None and old[1] & BLOCK_HAVE_UNDO:
            status |= BLOCK_HAVE_UNDO
            upos = old[5]
        self.entries[block_hash] = [height, status, n_tx, pos.file, pos.offset, upos, header_bytes]
        f = self.files.get(pos.file)
        if f is None or f[0] == 0:
            f = self.files[pos.file] = [0, 0, f[2] if f else 0, height, height, time, time]
        f[0] += 1
        f[1] = max(f[1], pos.offset + pos.size)
        f[3], f[4] = min(f[3], height), max(f[4], height)
        f[5], f[6] = min(f[5], time), max(f[6], time)
        self.last_file = max(self.last_file, pos.file)
        self.db.write([self._index_op(block_hash), self._file_op(pos.file), (b"l", self._x(_I32.pack(self.last_file)))])

    def set_undo(self, block_hash: bytes, file: int, undo_pos: int, undo_size: int) -> None:
        """The block was connected and its undo record written at rev`file`:`undo_pos`."""
        e = self.entries.get(block_hash)
        if e is None:
            return
        e[1] = (e[1] & ~BLOCK_VALID_MASK) | BLOCK_VALID_SCRIPTS | BLOCK_HAVE_UNDO
        e[3], e[5] = file, undo_pos
        f = self.files.setdefault(file, [0, 0, 0, 0, 0, 0, 0])
        f[2] = max(f[2], undo_pos + undo_size + 32)
        self.db.write([self._index_op(block_hash), self._file_op(file)])

    def set_failed(self, block_hash: bytes, failed: bool) -> None:
        e = self.entries.get(block_hash)
        if e is None:
            return
        e[1] = (e[1] | BLOCK_FAILED_VALID) if failed else (e[1] & ~(BLOCK_FAILED_VALID | BLOCK_FAILED_CHILD))
        self.db.write([self._index_op(block_hash)])

    def prune_file(self, fi: int) -> list[bytes]:
        """PruneOneBlockFile (src/validation.cpp:12208-12240): every block stored in blk`fi` loses
        its data and undo (status bits and positions cleared, the header stays), and the file's
        CBlockFileInfo is reset. Returns the blocks' hashes."""
        hit = [h for h, e in self.entries.items() if e[3] == fi and e[1] & (BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)]
        for h in hit:
            e = self.entries[h]
            e[1] &= ~(BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)
            e[3] = e[4] = e[5] = 0
        self.files[fi] = [0, 0, 0, 0, 0, 0, 0]
        self.db.write([self._index_op(h) for h in hit] + [self._file_op(fi)])
        return hit

    def rewrite(self, records) -> None:
        """After a full -reindex scan: records of (header bytes, pos, n_tx, height, hash, time)."""
        ops = [(k, None) for k, _ in self.db.items(b"b", b"c")] + [(k, None) for k, _ in self.db.items(b"f", b"g")]
        self.db.write(ops)
        self.entries.clear()
        self.files.clear()
        self.last_file = 0
        for hb, pos, ntx, height, h, t in records:
            self.append(hb, pos, ntx, height=height, block_hash=h, time=t)
        self.sync()

    def reindexing(self) -> bool:
        return self.db.get(b"R") is not None

    def set_reindexing(self, on: bool) -> None:
        self.db.write([(b"R", self._x(b"1") if on else None)], sync=True)

    def flag(self, name: str) -> bool | None:
        v = self.db.get(b"F" + bytes([len(name)]) + name.encode())
        return None if v is None else self._x(v) == b"1"

    def set_flag(self, name: str, value: bool) -> None:
        self.db.write([(b"F" + bytes([len(name)]) + name.encode(), self._x(b"1" if value else b"0"))], sync=True)

    def sync(self) -> None:
        self.db.write([(b"l", self._x(_I32.pack(self.last_file)))], sync=True)

    def close(self) -> None:
        if self.db is not None:
            self.sync()
            self.db.close()
            self.db = None


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
