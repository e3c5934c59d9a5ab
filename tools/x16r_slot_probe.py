#!/usr/bin/env python3
"""Per-slot latency of the batch X16R step kernel (x16r_step_all): for each of the 16 primitives, a
batch whose every header runs that primitive at all 16 steps (hashPrevBlock nibbles 48..63 set to
the slot), timed end to end; ms per step = batch time / 16. Prints one JSON line.

    python tools/x16r_slot_probe.py --n 16384
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["blake", "bmw", "groestl", "jh", "keccak", "skein", "luffa", "cubehash", "shavite", "simd", "echo",
         "hamsi", "fugue", "shabal", "whirlpool", "sha512"]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 14)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--hsaco", default=None, help="an x16r code object to use instead of kernels/x16r.hsaco")
    ap.add_argument("--slots", nargs="*", type=int, default=list(range(16)))
    a = ap.parse_args()

    import numpy as np
    import torch

    from nodexa_chain_core_amd.ops import runtime
    from nodexa_chain_core_amd.ops.x16r import selections, x16r_hash_batch

    if a.hsaco:  # A/B of a variant build: ops/x16r.py looks its kernels up through static_kernel
        co = runtime.load_code_object(a.hsaco)
        base_static = runtime.static_kernel
        runtime.static_kernel = lambda m, n: co.function(n) if m == "x16r" else base_static(m, n)

    rng = np.random.default_rng(11)
    base = rng.integers(0, 256, size=(a.n, 80), dtype=np.uint8)
    x16r_hash_batch(base[:256])
    torch.cuda.synchronize()
    out = {}
    for slot in a.slots:
        hdr = base.copy()
        hdr[:, 4:12] = (slot << 4) | slot  # nibbles 48..63 of hashPrevBlock
        assert (selections(hdr[:4]) == slot).all()
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            x16r_hash_batch(hdr)
            ts.append(time.perf_counter() - t)
        out[NAMES[slot]] = round(min(ts) / 16 * 1e3, 3)
    ts = []
    for _ in range(a.reps):  # the random batch (every slot mixed)
        t = time.perf_counter()
        x16r_hash_batch(base)
        ts.append(time.perf_counter() - t)
    print(json.dumps({"n": a.n, "hsaco": a.hsaco, "ms_per_step": out,
                      "mixed_hashes_per_s": round(a.n / min(ts))}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
