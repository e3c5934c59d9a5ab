#!/usr/bin/env python3
"""Throughput of batch X16R / X16RV2 on the GPU (ops/x16r.py, hip/kernels/x16r.hip) against the host's
native multi-threaded hashing of the same headers. Prints one JSON line.

    python tools/x16r_probe.py --n 65536 --reps 3
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", type=int, default=64)
    a = ap.parse_args()

    import numpy as np
    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.ops.x16r import x16r_hash_batch

    rng = np.random.default_rng(9)
    hdrs = rng.integers(0, 256, size=(a.n, 80), dtype=np.uint8)
    x16r_hash_batch(hdrs[:256])  # code object load
    torch.cuda.synchronize()
    res = {}
    for v2 in (False, True):
        times = []
        for _ in range(a.reps):
            t = time.perf_counter()
            got = x16r_hash_batch(hdrs, v2=v2)
            times.append(time.perf_counter() - t)
        bad = 0
        for i in range(0, a.n, max(1, a.n // a.check)):
            h = bytes(hdrs[i])
            bad += bytes(got[i]) != (_core.x16rv2 if v2 else _core.x16r)(h, h[4:36])
        res["x16rv2" if v2 else "x16r"] = {"s": round(min(times), 4), "hashes_per_s": round(a.n / min(times)),
                                          "mismatches": bad}
    # the nonce search (all nonces of a window run the same slots): a zero target scans every nonce
    from nodexa_chain_core_amd.ops.x16r import X16rSearcher

    srch = X16rSearcher(0, window=1 << 20)
    hdr = bytes(hdrs[0])
    srch.search(hdr, False, bytes(32), 0, 1 << 16)
    for v2 in (False, True):
        t = time.perf_counter()
        hit, n = srch.search(hdr, v2, bytes(32), 0, 1 << 22)
        dt = time.perf_counter() - t
        res[("x16rv2" if v2 else "x16r") + "_search"] = {"nonces": n, "s": round(dt, 4), "hashes_per_s": round(n / dt)}
    print(json.dumps({"n": a.n, **res}), flush=True)
    return 0 if all(r.get("mismatches", 0) == 0 for r in res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
