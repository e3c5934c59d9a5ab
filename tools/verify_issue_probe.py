#!/usr/bin/env python3
"""Where the resident verify pipeline's host time goes (ops/header_batch.ResidentHeaderVerifier.run).

Runs the 10k-header fixture through models/verify.process_batch_resident N times (fresh chain each
time, as bench.py does) with every HIP runtime call of the pipeline wrapped in a timer, and prints one
JSON line: per-stage medians (parse / plan / pack / issue / overlap / wait / accept) and, for the
issue stage, the time and count per runtime entry point plus the Python glue around them.

    python tools/verify_issue_probe.py --runs 30
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=30)
    a = ap.parse_args()

    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import process_batch_resident, resident_verifier
    from nodexa_chain_core_amd.ops import header_batch as HB

    fix = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "data",
                       "testnet_mixed_10k.hdr")
    params, headers = synthetic.load(fix)
    raw = open(fix, "rb").read()
    act = params.kawpow_activation_time
    adjusted = headers[-1].time + 3600

    def once():
        chain = _core.HeaderChain(params)
        t = time.perf_counter()
        b = _core.HeaderBatch.from_bytes(raw, act)
        parse = time.perf_counter() - t
        r = process_batch_resident(chain, b, adjusted, device=0)
        return time.perf_counter() - t, parse, r

    once()  # DAGs, program tables, code objects
    torch.cuda.synchronize()

    # time every runtime call made while the pipeline issues
    v = resident_verifier(0)
    h = v.h
    calls = collections.defaultdict(lambda: [0, 0.0])

    class Timed:
        def __init__(self, inner):
            self._inner = inner

        def __getattr__(self, name):
            fn = getattr(self._inner, name)
            if not callable(fn):
                return fn

            def wrap(*args, **kw):
                t = time.perf_counter()
                try:
                    return fn(*args, **kw)
                finally:
                    c = calls[name]
                    c[0] += 1
                    c[1] += time.perf_counter() - t
            return wrap

    totals, stages = [], collections.defaultdict(list)
    for timed in (False, True):
        v.h = Timed(h) if timed else h
        for _ in range(a.runs):
            dt, parse, r = once()
            if not timed:
                totals.append(dt)
                stages["parse_ms"].append(parse * 1e3)
                for k in ("pack_ms", "issue_ms", "overlap_ms", "wait_ms", "accept_ms", "device_ms"):
                    stages[k].append(r[k])
    v.h = h
    # the host parts of the overlap and accept stages, each on its own (fresh batch / chain)
    parts = collections.defaultdict(list)
    for _ in range(a.runs):
        chain = _core.HeaderChain(params)
        b = _core.HeaderBatch.from_bytes(raw, act)
        t = time.perf_counter()
        b.materialize()
        parts["materialize_ms"].append((time.perf_counter() - t) * 1e3)
        r = process_batch_resident(_core.HeaderChain(params), _core.HeaderBatch.from_bytes(raw, act), adjusted, device=0)
        hashes = v.early_host.numpy()[:len(headers) * 32].copy()
        bits = v.early_host.numpy()[len(headers) * 32:len(headers) * 36].view("<u4").copy()
        t = time.perf_counter()
        prep = chain.prepare_batch(b, adjusted, hashes, bits)
        parts["prepare_ms"].append((time.perf_counter() - t) * 1e3)
        t = time.perf_counter()
        chain.commit_batch(prep, len(headers))
        parts["commit_ms"].append((time.perf_counter() - t) * 1e3)
    out_parts = {k: round(statistics.median(x), 3) for k, x in parts.items()}
    out = {"host_parts_ms": out_parts,"runs": a.runs, "median_ms": round(statistics.median(totals) * 1e3, 3),
           "headers_per_s": round(len(headers) / statistics.median(totals)),
           "stages_ms": {k: round(statistics.median(x), 3) for k, x in stages.items()},
           "runtime_calls_per_run": {k: {"n": c[0] // a.runs, "us": round(c[1] / a.runs * 1e6, 1)}
                                     for k, c in sorted(calls.items(), key=lambda kv: -kv[1][1])}}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
