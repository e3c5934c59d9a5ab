#!/usr/bin/env python3
"""Which Equihash device-side caps fire (per instance): segment/staging drops per level, chain
truncations, candidate counts — and how many instances the host re-solved."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch

    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    s = EquihashSolver(num_inst=8, device=0, engine="ps")
    h = s.h
    for b in range(3):
        inputs = [bytes(80) + (b * 8 + i).to_bytes(32, "little") for i in range(8)]
        t0 = time.time()
        s.launch(inputs)
        torch.cuda.synchronize()
        st = s.stats_buf.view(8, h.EQP_STATS).cpu().tolist()
        cands = s.cands.view(8, -1)[:, 0].cpu().tolist()
        sols = s.sols.view(8, -1)[:, 0].cpu().tolist()
        before = s.fallbacks
        out = s.collect()
        print({"batch": b, "stats": st, "cands": cands, "sols": sols, "fallbacks": s.fallbacks - before,
               "found": [len(x) for x in out], "s": round(time.time() - t0, 3)}, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
