#!/usr/bin/env python3
"""kawpow_verify_waves against probe variants (tools/verify_waves_variants.hip, compiled here to
gpurun_out/pv.hsaco by the caller): the 10k fixture's resident run is captured once (every
launch_kawpow_verify_waves argument), then each variant replays the captured launches, timed with
hip events (median of --reps), and its full hashes are compared with the shipping kernel's.
Prints one JSON line per kernel.

    python tools/verify_waves_probe.py --hsaco gpurun_out/pv.hsaco --variants 0 1 2 3 4 5
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
    ap.add_argument("--hsaco", required=True)
    ap.add_argument("--variants", nargs="*", type=int, default=[0, 1, 2, 3, 4, 5])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()

    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import process_batch_resident, resident_verifier
    from nodexa_chain_core_amd.ops import runtime

    fix = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "data",
                       "testnet_mixed_10k.hdr")
    params, headers = synthetic.load(fix)
    raw = open(fix, "rb").read()
    act = params.kawpow_activation_time
    v = resident_verifier(0)
    h = v.h
    calls = []

    class Capture:
        def __getattr__(self, name):
            fn = getattr(h, name)
            if name != "launch_kawpow_verify_waves":
                return fn

            def wrap(*args):
                calls.append(args)
                return fn(*args)
            return wrap

    v.h = Capture()
    try:
        process_batch_resident(_core.HeaderChain(params), _core.HeaderBatch.from_bytes(raw, act),
                               headers[-1].time + 3600, device=0)
    finally:
        v.h = h
    torch.cuda.synchronize()
    # outputs: (out pointer, jobs) of each captured launch -> views of v.full
    base = v.full.data_ptr()
    regions = [((c[11] - base) // 4, c[8]) for c in calls]

    def snapshot():
        return [v.full[o:o + 16 * n].clone() for o, n in regions]

    co = runtime.load_code_object(a.hsaco)
    kernels = [("kawpow_verify_waves", v.k_waves)] + [(f"pv_waves_{i}", co.function(f"pv_waves_{i}")) for i in a.variants]
    s = runtime.current_stream_handle()
    ref = None
    for name, k in kernels:
        times = []
        for rep in range(a.reps + 1):
            v.full.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for c in calls:
                h.launch_kawpow_verify_waves(k, *c[1:12], s)
            e1.record()
            e1.synchronize()
            if rep:
                times.append(e0.elapsed_time(e1) * 1e3)
        got = snapshot()
        if ref is None:
            ref = got
        same = all(torch.equal(x, y) for x, y in zip(got, ref))
        print(json.dumps({"kernel": name, "launches": len(calls), "jobs": sum(n for _, n in regions),
                          "median_us": round(statistics.median(times), 1), "min_us": round(min(times), 1),
                          "bit_exact_vs_shipping": same}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
