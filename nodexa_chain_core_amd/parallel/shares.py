"""Winning-share all-gather over RCCL (collective #2).

Each rank's search kernel appends shares to a fixed-size ring
(KawpowResults, 4.6 KB). Right after the kernel, on the same stream, the rings
are all-gathered into a [world, ring] tensor so rank 0 (the node / pool
front-end) sees every GPU's shares without any host round-trip per step. The
collective is latency-bound (tens of µs over xGMI), never bandwidth-bound.
"""
from __future__ import annotations

import struct

import torch
import torch.distributed as dist

from . import world as W

# KawpowResults layout (hip/kernels/kernel_params.h): u32 count, 3 pad, then
# shares of {u64 nonce, u32 mix[8], u32 final[8]}.
SHARE_FMT = "<Q8I8I"
SHARE_SIZE = struct.calcsize(SHARE_FMT)
RING_HEADER = 16


def parse_ring(raw: bytes, max_shares: int, base: int = 0) -> list[tuple[int, bytes, bytes]]:
    """(nonce, mix, final) entries of one result ring (count clamped to the ring size)."""
    count = struct.unpack_from("<I", raw, base)[0]
    out = []
    for i in range(min(count, max_shares)):
        vals = struct.unpack_from(SHARE_FMT, raw, base + RING_HEADER + i * SHARE_SIZE)
        out.append((vals[0], struct.pack("<8I", *vals[1:9]), struct.pack("<8I", *vals[9:17])))
    return out


class ShareGather:
    """All-gather of every rank's share ring into one [world x ring] device tensor.

    `ShareGather(searcher)` for an ops.kawpow.KawpowSearcher, or
    `ShareGather(results=tensor, max_shares=n)` for any ring-shaped int32 tensor."""

    def __init__(self, searcher=None, *, results: torch.Tensor | None = None, max_shares: int | None = None):
        self.results = searcher.results if searcher is not None else results
        self.max_shares = searcher.h.KAWPOW_MAX_SHARES if searcher is not None else int(max_shares)
        self.w = W.get()
        n = self.results.numel()
        self.gathered = torch.zeros(self.w.world_size * n, dtype=self.results.dtype, device=self.results.device)
        self._views = list(self.gathered.view(self.w.world_size, n).unbind(0))

    def enqueue(self) -> None:
        """Queue the gather after the last search launch (no host sync on RCCL)."""
        if not self.w.distributed:
            self.gathered.copy_(self.results, non_blocking=True)
        elif self.w.backend == "nccl":
            dist.all_gather_into_tensor(self.gathered, self.results, group=self.w.group)
        else:
            dist.all_gather(self._views, self.results, group=self.w.group)

    def collect(self):
        from ..ops.kawpow import Share

        raw = self.gathered.cpu().numpy().tobytes()
        per = self.results.numel() * self.results.element_size()
        out = [Share(n, mix, fin) for r in range(self.w.world_size)
               for n, mix, fin in parse_ring(raw, self.max_shares, r * per)]
        out.sort(key=lambda s: s.nonce)
        return out
