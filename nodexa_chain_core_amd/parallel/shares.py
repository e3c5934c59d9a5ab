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

from ..ops.kawpow import SHARE_FMT, SHARE_SIZE, KawpowSearcher, Share
from . import world as W


class ShareGather:
    def __init__(self, searcher: KawpowSearcher):
        self.s = searcher
        self.w = W.get()
        n = searcher.results.numel()
        self.gathered = torch.zeros(self.w.world_size * n, dtype=torch.int32, device=searcher.device)

    def enqueue(self) -> None:
        """Queue the gather after the last search launch (no host sync)."""
        if self.w.distributed:
            dist.all_gather_into_tensor(self.gathered, self.s.results)
        else:
            self.gathered.copy_(self.s.results, non_blocking=True)

    def collect(self) -> list[Share]:
        raw = self.gathered.cpu().numpy().tobytes()
        per = self.s.results.numel() * 4
        max_shares = self.s.h.KAWPOW_MAX_SHARES
        out: list[Share] = []
        for r in range(self.w.world_size):
            base = r * per
            count = struct.unpack_from("<I", raw, base)[0]
            for i in range(min(count, max_shares)):
                vals = struct.unpack_from(SHARE_FMT, raw, base + 16 + i * SHARE_SIZE)
                out.append(Share(vals[0], struct.pack("<8I", *vals[1:9]), struct.pack("<8I", *vals[9:17])))
        out.sort(key=lambda s: s.nonce)
        return out
