#!/usr/bin/env python3
"""Throughput of the classic Ethash hashimoto kernels (hip/kernels/ethash_hashimoto.hip: seed, mix,
final; `--kernels` picks the mix kernel variants) over a
resident DAG: random (header hash, nonce) jobs generated on the device, timed launches (hip
events), the first results re-checked against the host's ethash_hash. Prints one JSON line.

    python tools/hashimoto_probe.py --epoch 384 --jobs 4194304 --reps 5

(r5i compared 1 / 2 / 4 / 8 hashes per row with extra `ethash_mix_batch_hN` entry points that were
removed after it; EH_HASHES=2 ships.)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--epoch", type=int, default=384)
    ap.add_argument("--jobs", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=32)
    ap.add_argument("--kernels", nargs="*", default=["ethash_mix_batch"])
    a = ap.parse_args()

    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.ops import runtime
    from nodexa_chain_core_amd.ops.ethash import DeviceEpoch

    torch.cuda.set_device(0)
    e = DeviceEpoch(a.epoch, device=0, ctx=_core.get_epoch_context(a.epoch))
    e.build()
    torch.cuda.synchronize()
    n = a.jobs
    g = torch.Generator(device="cuda:0").manual_seed(5)
    jobs = torch.randint(-2**31, 2**31 - 1, (n, 12), dtype=torch.int32, device="cuda:0", generator=g)
    jobs[:, 10:] = 0
    out = torch.empty(n * 16, dtype=torch.int32, device="cuda:0")
    h = runtime.hip()
    from nodexa_chain_core_amd.ops.ethash import EH_HASHES

    s = runtime.current_stream_handle()
    bad_total = 0
    seeds = torch.empty(n * 16, dtype=torch.int32, device="cuda:0")
    k_seed = runtime.static_kernel("ethash_hashimoto", "ethash_seed_batch")
    k_final = runtime.static_kernel("ethash_hashimoto", "ethash_final_batch")
    for name in a.kernels:
        k = runtime.static_kernel("ethash_hashimoto", name)
        per_row = EH_HASHES if name == "ethash_mix_batch" else int(name.rsplit("_h", 1)[1])
        out.zero_()
        times = []
        for _ in range(a.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.launch_ethash_hash_batch(k_seed, k, k_final, e.dag.data_ptr(), e.full_items, jobs.data_ptr(), n,
                                       out.data_ptr(), seeds.data_ptr(), s, per_row)
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3)
        times = times[1:]
        idx = list(range(a.check)) + list(range(n - a.check, n))  # both ends of the batch
        jb = jobs.cpu().numpy().tobytes()
        res = out.cpu().numpy().tobytes()
        bad = 0
        for i in idx:
            hh = jb[i * 48:i * 48 + 32]
            nonce = int.from_bytes(jb[i * 48 + 32:i * 48 + 40], "little")
            f, m = _core.ethash_hash(e.ctx, hh, nonce)
            bad += (res[i * 64:i * 64 + 32], res[i * 64 + 32:i * 64 + 64]) != (m, f)
        bad_total += bad
        med = statistics.median(times)
        print(json.dumps({"kernel": name, "hashes_per_row": per_row, "epoch": a.epoch,
                          "dag_gib": round(e.dag_bytes / 2**30, 2), "jobs": n, "median_s": round(med, 5),
                          "mhs": round(n / med / 1e6, 1), "dag_gbps": round(n * 64 * 128 / med / 1e9, 1),
                          "checked": len(idx), "mismatches": bad}), flush=True)
    return 1 if bad_total else 0


if __name__ == "__main__":
    sys.exit(main())
