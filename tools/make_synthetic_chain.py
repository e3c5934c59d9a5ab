#!/usr/bin/env python3
"""Mine a synthetic KawPow testnet header chain (models/synthetic.py) to a file.

    python tools/make_synthetic_chain.py --n 10000 --out tests/data/testnet_kawpow_10k.hdr [--backend gpu] [--equihash 1000]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--out", required=True)
    ap.add_argument("--backend", choices=["cpu", "gpu"], default="cpu")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--equihash", type=int, default=0, help="Equihash-extension headers mined after the KawPow ones")
    a = ap.parse_args()
    from nodexa_chain_core_amd.models import synthetic

    t0 = time.time()
    params, headers = synthetic.build_chain(
        a.n, a.equihash, backend=a.backend, seed=a.seed,
        progress=lambda i: print(f"[synthetic] {i} headers, {time.time() - t0:.0f}s", flush=True))
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    synthetic.save(a.out, params, headers)
    bits = sorted({h.bits for h in headers})
    print(f"[synthetic] wrote {len(headers)} headers to {a.out} in {time.time() - t0:.0f}s; "
          f"{len(bits)} distinct nBits, min {hex(bits[0])} max {hex(bits[-1])}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
