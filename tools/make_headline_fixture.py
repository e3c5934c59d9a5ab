#!/usr/bin/env python3
"""Mine the headline-epoch header fixture of BASELINE config 5 on a GPU.

10,000 testnet-rule headers at heights 2,880,000-2,889,999 (KawPow epochs 384 -> 385 at 2,887,500,
4 GiB DAGs, 64 MiB light caches), the last `--equihash` of them Equihash(200,9) extension headers,
built on a 181-header anchor (models/synthetic.make_anchor: the stored index a node has below the
fixture; DarkGravityWave reads its 180 last headers). KawPow nonces are searched on the resident
DAG (ops/verify.DagNonceScanner), Equihash solutions by the gfx950 solver; every header is accepted
into a HeaderChain as it is built.

    python tools/make_headline_fixture.py --out gpurun_out/fixture/testnet_mixed_e384_10k.hdr
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--first-height", type=int, default=2_880_000)
    ap.add_argument("--headers", type=int, default=10_000)
    ap.add_argument("--equihash", type=int, default=170)
    ap.add_argument("--seed", type=int, default=384)
    a = ap.parse_args()

    from nodexa_chain_core_amd.models import synthetic

    t0 = time.time()

    def progress(i):
        print(f"[fixture] {i}/{a.headers} headers, {time.time() - t0:.0f}s", flush=True)

    params, hs, anchor = synthetic.build_chain(a.headers - a.equihash, a.equihash, network="test", backend="gpu",
                                               seed=a.seed, first_height=a.first_height, progress=progress)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    synthetic.save(a.out, params, hs, anchor)
    print(f"[fixture] {len(hs)} headers, heights {hs[0].height}-{hs[-1].height}, written to {a.out} "
          f"in {time.time() - t0:.0f}s", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
