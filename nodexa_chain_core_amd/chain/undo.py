"""Block undo records in rev?????.dat files.

Parity: UndoWriteToDisk / UndoReadFromDisk (src/validation.cpp): a record is
`message start (4) | u32 size | CBlockUndo | sha256d(previous block hash || CBlockUndo)`; the
CBlockUndo bytes come from the native core (`_core.connect_block`, the reference's compressed coin
encoding). Files roll over at 128 MiB like blk files (MAX_BLOCKFILE_SIZE). Where each block's
record lives is kept in an append-only `blocks/undo.idx` (block hash, file, offset, size), the
counterpart of the undo position in CDiskBlockIndex; a torn last entry is ignored on load.

A second store with prefix "aun" holds the asset undo records (the asset journal of each block,
csrc/chain/assets.hpp), the role of CBlockAssetUndo in the reference's assets database.
"""
from __future__ import annotations

import hashlib
import os
import struct

MAX_FILE = 128 * 1024 * 1024
_IDX = struct.Struct("<32sIII")


def _sha256d(b: bytes) -> bytes:
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()


class UndoStore:
    def __init__(self, bdir: str, magic: bytes, prefix: str = "rev"):
        self.bdir = bdir
        self.prefix = prefix
        self.magic = bytes(magic)
        self.pos: dict[bytes, tuple[int, int, int]] = {}
        self._mem: dict[bytes, bytes] = {}  # memory-only store (no datadir)
        self.file = 0
        self._idx = None
        if bdir is None:
            return
        os.makedirs(bdir, exist_ok=True)
        idx = os.path.join(bdir, "undo.idx" if prefix == "rev" else f"{prefix}.idx")
        if os.path.exists(idx):
            with open(idx, "rb") as f:
                data = f.read()
            present: dict[int, bool] = {}
            for off in range(0, len(data) - len(data) % _IDX.size, _IDX.size):
                h, fi, fo, size = _IDX.unpack_from(data, off)
                if fi not in present:
                    present[fi] = os.path.exists(self._path(fi))
                if not present[fi]:  # a pruned file: its records are gone
                    continue
                self.pos[h] = (fi, fo, size)
                self.file = max(self.file, fi)
            if len(data) % _IDX.size:  # torn tail from a crash: cut it
                with open(idx, "r+b") as f:
                    f.truncate(len(data) - len(data) % _IDX.size)
        self._idx = open(idx, "ab")

    def _path(self, fi: int) -> str:
        return os.path.join(self.bdir, f"{self.prefix}{fi:05d}.dat")

    def write(self, block_hash: bytes, prev_hash: bytes, undo: bytes, file: int | None = None):
        """Append the record; returns its (file, data offset, size). With `file` (the block's blk
        file number) it goes to rev`file`, as the reference keeps a block's undo data beside it
        (CBlockIndex::nFile serves both); otherwise files roll over at MAX_FILE."""
        if self.bdir is None:
            self._mem[block_hash] = undo
            return None
        if file is not None:
            self.file = max(self.file, file)
            path = self._path(file)
            size = os.path.getsize(path) if os.path.exists(path) else 0
        else:
            file = self.file
            path = self._path(file)
            size = os.path.getsize(path) if os.path.exists(path) else 0
            if size + len(undo) + 40 > MAX_FILE and size > 0:
                self.file = file = file + 1
                path, size = self._path(file), 0
        rec = self.magic + struct.pack("<I", len(undo)) + undo + _sha256d(prev_hash + undo)
        with open(path, "ab") as f:
            f.write(rec)
        self.pos[block_hash] = (file, size + 8, len(undo))
        self._idx.write(_IDX.pack(block_hash, file, size + 8, len(undo)))
        self._idx.flush()
        return self.pos[block_hash]

    def drop_file(self, fi: int) -> int:
        """Pruning: forget every record of file `fi` and delete it; returns the bytes freed."""
        for h in [h for h, p in self.pos.items() if p[0] == fi]:
            del self.pos[h]
        if self.bdir is None:
            return 0
        path = self._path(fi)
        try:
            n = os.path.getsize(path)
            os.remove(path)
            return n
        except OSError:
            return 0

    def adopt(self, block_hash: bytes, file: int, offset: int) -> bool:
        """Register a record another index located (a reference blocks/index 'b' record's
        nUndoPos); the size comes from the record's framing. False if the framing is wrong."""
        path = self._path(file)
        try:
            with open(path, "rb") as f:
                f.seek(offset - 8)
                head = f.read(8)
        except OSError:
            return False
        if len(head) != 8 or head[:4] != self.magic:
            return False
        self.pos[block_hash] = (file, offset, struct.unpack("<I", head[4:])[0])
        self.file = max(self.file, file)
        return True

    def read(self, block_hash: bytes, prev_hash: bytes) -> bytes | None:
        if self.bdir is None:
            return self._mem.get(block_hash)
        p = self.pos.get(block_hash)
        if p is None:
            return None
        fi, off, size = p
        with open(self._path(fi), "rb") as f:
            f.seek(off - 8)
            head = f.read(8)
            undo = f.read(size)
            check = f.read(32)
        if head[:4] != self.magic or struct.unpack("<I", head[4:])[0] != size:
            raise IOError("undo record header mismatch")
        if _sha256d(prev_hash + undo) != check:
            raise IOError("undo record checksum mismatch")
        return undo

    def close(self) -> None:
        if self._idx is not None:
            self._idx.close()
            self._idx = None
