#!/usr/bin/env python3
"""Which Equihash device-side caps fire on the bench's inputs (the header + (rank, batch, slot)
nonces of bench.py): per-instance truncation counters of every re-solved instance."""
import os
import struct
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.chain.header import BlockHeader
    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    hdr = BlockHeader(version=0x20000000, prev=_core.sha256d(b"nodexa-bench-prev"),
                      merkle_root=_core.sha256d(b"nodexa-bench-merkle"), time=1_700_000_000,
                      bits=0x1b00ffff, height=384 * 7500 + 123)
    s = EquihashSolver(num_inst=8, device=0)
    t0 = time.time()
    n = 0
    for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 24):
        inputs = [hdr.kawpow_input() + struct.pack("<QQQQ", 0, i, j, 0xE9) for j in range(8)]
        n += sum(len(x) for x in s.solve(inputs))
        st = s.stats_buf.view(8, s.h.EQP_STATS).cpu()
        print({"batch": i, "largest_bucket": st[:, s.h.EQP_STAT_STAGE_MAX].tolist(),
               "stage_dropped": st[:, s.h.EQP_STAT_STAGE].tolist(), "segment_dropped": st[:, :9].sum(1).tolist()},
              flush=True)
    torch.cuda.synchronize()
    print({"solutions": n, "s": round(time.time() - t0, 3), "fallbacks": s.fallbacks, "log": s.fallback_log},
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
