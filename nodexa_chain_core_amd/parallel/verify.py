"""Batch header verification across ranks: one process per GPU, results over RCCL.

Every rank holds the same header batch (a P2P `headers` message, a -loadblock file, the
10k-header fixture). The cheap native prepare pass (job records, boundaries, mix-only
prefilter) runs on every rank; the full-ProgPoW candidates are split into contiguous
slices, each rank hashes its slice on its own GPU (ops/verify.gpu_hash_jobs), and the
64-byte result rows are all-gathered device to device (all_gather_into_tensor: RCCL over
xGMI, one collective of n x 64 bytes) so every rank ends with the full result and can run
the contextual stage itself. CPU rehearsals (gloo) hash with the C++ golden model.

Parity: the reference verifies a header batch serially on one thread under cs_main
(src/validation.cpp:12017-12035); it has no multi-device path.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ..models.verify import _cpu_rows, _verify_native
from . import world as W


def _sharded_rows(jobs: np.ndarray, mode: str) -> np.ndarray:
    w = W.get()
    m = len(jobs)
    per = -(-m // w.world_size) if m else 0
    mine = jobs[w.rank * per: min(m, (w.rank + 1) * per)]
    if w.device.type == "cuda":
        from ..ops.verify import gpu_hash_jobs

        local = gpu_hash_jobs(mine, device=w.device.index, mode=mode) if len(mine) else np.zeros((0, 64), np.uint8)
    else:
        local = _cpu_rows(mine, 0) if len(mine) else np.zeros((0, 64), np.uint8)
    if not w.collective:  # one rank: its rows are the batch's, no round trip through the device
        return np.ascontiguousarray(local)[:m]
    buf = torch.zeros((per, 64), dtype=torch.uint8, device=w.device)
    if len(local):
        buf[:len(local)] = torch.from_numpy(np.ascontiguousarray(local)).to(w.device)
    out = torch.empty((per * w.world_size, 64), dtype=torch.uint8, device=w.device)
    dist.all_gather_into_tensor(out, buf, group=w.group)
    return out.cpu().numpy()[:m]


def verify_headers_distributed(params, headers, mode: str = "auto") -> list[dict]:
    """verify_headers with the full-hash work split over all ranks (same result on every rank)."""
    from .. import core

    _core = core()
    act = params.kawpow_activation_time
    hs = [h if isinstance(h, _core.BlockHeader) else _core.BlockHeader.deserialize(h.serialize(act), act)
          for h in headers]
    w = W.get()
    gpus = [w.device.index] if w.device.type == "cuda" else None
    return _verify_native(params, hs, gpus, 0, mode, rows_fn=lambda jobs: _sharded_rows(jobs, mode))
