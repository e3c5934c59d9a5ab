#!/usr/bin/env python3
"""GPU batch ECDSA verification throughput (hip/kernels/secp256k1_verify.hip): device time per
batch (hip events) for several batch sizes, plus the host golden model's rate for comparison.
Signatures are 2048 distinct valid ones tiled to the batch size (the kernel's work does not
depend on duplicates). Prints JSON lines."""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="*", default=[65536, 262144, 1048576])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.ops import runtime, secp

    rng = random.Random(1)
    base = []
    while len(base) < 2048:
        k = rng.randbytes(32)
        if _core.secp_seckey_valid(k):
            m = rng.randbytes(32)
            base.append((_core.secp_pubkey_create(k, len(base) % 4 != 0), _core.secp_sign(m, k), m))
    t = time.perf_counter()
    for p, s, m in base[:256]:
        assert _core.secp_verify(p, s, m)
    host_rate = 256 / (time.perf_counter() - t)
    print(json.dumps({"host_golden_verifies_per_s_1core": round(host_rate, 1)}), flush=True)
    assert all(secp.verify_batch(base[:1024], device=0))
    h = runtime.hip()
    dev = torch.device("cuda", 0)
    kern = runtime.static_kernel("secp256k1_verify", "secp_verify_batch")
    packed = bytearray(_core.secp_pack_jobs(base))
    gtab = secp._gen_table(dev)
    for n in a.sizes:
        reps = (n + len(base) - 1) // len(base)
        jobs = torch.frombuffer(packed * reps, dtype=torch.int32).to(dev)
        out = torch.empty(reps * len(base), dtype=torch.int32, device=dev)
        times = []
        for _ in range(a.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.launch_secp_verify(kern, jobs.data_ptr(), n, gtab.data_ptr(), out.data_ptr(),
                                 runtime.current_stream_handle())
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3)
        ok = int((out[:n] == 1).sum().item())
        best = min(times[1:])
        print(json.dumps({"batch": n, "device_s": round(best, 5), "verifies_per_s": round(n / best, 1),
                          "valid": ok}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
