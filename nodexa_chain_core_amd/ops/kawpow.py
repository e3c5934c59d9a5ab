"""KawPow nonce search and batch hashing on one MI355X.

Wraps the per-period gfx950 kernel (hip/kernels/kawpow_search.hip + the
generated program, see ops/jit.py). Reference behaviour: progpow::search /
hash (src/crypto/ethash/lib/ethash/progpow.cpp:357-429, 567-579); unlike the
reference's "first nonce wins" scan, one launch evaluates a whole nonce window
and returns every share whose final hash passes the 64-bit target prefix; the
host then re-checks each share bit-exactly (`Share.verify_host`).

Hashes here are in ethash storage order (the bytes progpow consumes); the
node-level byte reversal of the SHA256d header hash lives in chain/header.py.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import torch

from .. import _core
from . import jit, runtime
from ..utils.trace import traced
from .ethash import DeviceEpoch

SHARE_FMT = "<Q8I8I"
SHARE_SIZE = struct.calcsize(SHARE_FMT)


@dataclass
class Share:
    nonce: int
    mix_hash: bytes   # 32 bytes, storage order
    final_hash: bytes  # 32 bytes, storage order

    def verify_host(self, block_number: int, header_hash: bytes, boundary: bytes | None = None) -> bool:
        """Mix-only recomputation (cheap: the final keccak from the GPU's own mix) + optional full
        256-bit boundary check. A wrong DAG gather or program would pass this; `verify_full` not."""
        fin = _core.kawpow_hash_no_verify(block_number, header_hash, self.mix_hash, self.nonce)
        if fin != self.final_hash:
            return False
        return boundary is None or _core.hash_le(fin, boundary)

    def verify_full(self, block_number: int, header_hash: bytes, boundary: bytes | None = None, ctx=None) -> bool:
        """Full light-mode KawPow on the host (progpow::verify, src/crypto/ethash/lib/ethash/
        progpow.cpp:431-495): recompute mix and final from the epoch's light cache and require both
        to equal what the GPU reported (+ optional 256-bit boundary check)."""
        ctx = ctx if ctx is not None else _core.get_epoch_context(block_number // _core.EPOCH_LENGTH)
        fin, mix = _core.kawpow_hash(ctx, block_number, header_hash, self.nonce)
        if fin != self.final_hash or mix != self.mix_hash:
            return False
        return boundary is None or _core.hash_le(fin, boundary)


def parse_results(raw: bytes, max_shares: int) -> tuple[list[Share], int, int]:
    """(shares sorted by nonce, appended count, skipped workgroups) of one KawpowResults ring."""
    count, skipped = struct.unpack_from("<II", raw, 0)
    shares = []
    for i in range(min(count, max_shares)):
        vals = struct.unpack_from(SHARE_FMT, raw, 16 + i * SHARE_SIZE)
        shares.append(Share(vals[0], struct.pack("<8I", *vals[1:9]), struct.pack("<8I", *vals[9:17])))
    shares.sort(key=lambda s: s.nonce)
    return shares, count, skipped


def target_prefix(boundary: bytes) -> int:
    """Upper 64 bits (big-endian) of a 32-byte boundary, rounded so the GPU
    prefix test never rejects a hash the full compare would accept."""
    return int.from_bytes(boundary[:8], "big")


class KawpowSearcher:
    """Search / hash engine for one (device, epoch, period)."""

    def __init__(self, epoch_dev: DeviceEpoch, block_number: int, prefetch_next: bool = False):
        self.prefetch_next = prefetch_next
        self.epoch_dev = epoch_dev
        self.device = epoch_dev.device
        self.h = runtime.hip()
        self.block_number = -1
        self.period = -1
        self.kernel = None
        self.hash_kernel = None
        self._scratch: torch.Tensor | None = None
        nbytes = self.h.sizeof_results()
        with torch.cuda.device(self.device):
            self.results = torch.zeros(nbytes // 4, dtype=torch.int32, device=self.device)
            self.results_host = torch.zeros(nbytes // 4, dtype=torch.int32).pin_memory()
        self.set_block(block_number)

    def set_block(self, block_number: int) -> None:
        if block_number // _core.EPOCH_LENGTH != self.epoch_dev.epoch:
            raise ValueError(f"block {block_number} is not in epoch {self.epoch_dev.epoch}")
        period = block_number // 3
        if period != self.period:
            defines = jit.defines_for(self.epoch_dev.dag_bytes)
            with torch.cuda.device(self.device):
                path = jit.get(period, defines)
                co = runtime.load_code_object(path, key=path)
                self.kernel = co.function("kawpow_search")
                self.hash_kernel = co.function("kawpow_hash_batch")
            self.period = period
            if self.prefetch_next:
                jit.prefetch(period + 1, defines)  # next period compiles while this one mines
        self.block_number = block_number

    @property
    def block(self) -> int:
        """Threads per workgroup of the loaded variant = the nonce granularity of a launch."""
        return int(self.kernel.max_threads)

    # ------------------------------------------------------------------
    def launch(self, header_hash: bytes, start_nonce: int, num_nonces: int, target64: int,
               stream: int | None = None, results: torch.Tensor | None = None, gen_word: int = 0,
               generation: int = 0) -> None:
        """Queue one search window on `stream` (no host sync). `results`: the share ring to append
        to (default: this searcher's own; the caller clears a ring it passes). `gen_word`: host-mapped
        generation word; workgroups that start after it moved past `generation` search nothing."""
        if num_nonces % self.block:
            raise ValueError(f"num_nonces must be a multiple of {self.block}")
        with torch.cuda.device(self.device):
            s = runtime.current_stream_handle() if stream is None else stream
            scratch = self.scratch(num_nonces)
            if results is None:
                results = self.results
                results[:4].zero_()
            self.h.launch_kawpow_search(self.kernel, self.epoch_dev.dag.data_ptr(), self.epoch_dev.items2048,
                                        results.data_ptr(), header_hash, start_nonce, target64, num_nonces, s,
                                        scratch.data_ptr(), scratch.numel() * 4, gen_word, generation)

    def scratch(self, num_nonces: int) -> torch.Tensor:
        """Per-nonce digest parking space (8 words/nonce) for the launch; grown on demand.
        Reused across launches: kernels on one stream are ordered."""
        need = num_nonces * 8
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.int32, device=self.device)
        return self._scratch

    def collect(self) -> list[Share]:
        """Copy the share ring back (synchronises the current stream)."""
        with torch.cuda.device(self.device):
            self.results_host.copy_(self.results, non_blocking=False)
        return parse_results(self.results_host.numpy().tobytes(), self.h.KAWPOW_MAX_SHARES)[0]

    @traced("kawpow.search")
    def search(self, header_hash: bytes, start_nonce: int, num_nonces: int, boundary: bytes) -> list[Share]:
        """All shares in [start, start+num) with final <= boundary (bit-exact, host-checked).
        The launch is rounded up to whole workgroups; shares past the window are dropped."""
        padded = -(-num_nonces // self.block) * self.block
        self.launch(header_hash, start_nonce, padded, target_prefix(boundary))
        end = start_nonce + num_nonces
        return [s for s in self.collect() if s.nonce < end and _core.hash_le(s.final_hash, boundary)]

    def hash_batch(self, header_hashes: list[bytes], nonces: list[int]) -> list[tuple[bytes, bytes]]:
        """(final, mix) for each (header, nonce) at this searcher's block height."""
        n = len(nonces)
        if n == 0:
            return []
        job = struct.Struct("<8IQII")
        buf = bytearray(job.size * n)
        for i, (hh, nonce) in enumerate(zip(header_hashes, nonces)):
            job.pack_into(buf, i * job.size, *struct.unpack("<8I", hh), nonce, self.block_number, 0)
        with torch.cuda.device(self.device):
            jobs = torch.frombuffer(buf, dtype=torch.uint8).to(self.device)
            out = torch.empty(n * 16, dtype=torch.int32, device=self.device)
            self.h.launch_kawpow_hash_batch(self.hash_kernel, self.epoch_dev.dag.data_ptr(), self.epoch_dev.items2048,
                                            jobs.data_ptr(), n, out.data_ptr(), runtime.current_stream_handle())
            raw = out.cpu().numpy().tobytes()
        res = []
        for i in range(n):
            mix = raw[i * 64:i * 64 + 32]
            fin = raw[i * 64 + 32:i * 64 + 64]
            res.append((fin, mix))
        return res
