"""Where the light-mode batch verify spends its time (bench.py `verify_headers.light`).

Runs the bench's light verify of a 10k-header fixture (no DAG resident) a few times with host
timers around the stages of ops/verify.gpu_hash_jobs (per epoch group: program table + uploads,
launch, read-back) and the whole PoW stage, and prints one JSON line per run. Under
`rocprofv3 --kernel-trace` the kernel timeline shows whether the epoch groups overlap.

  python tools/verify_light_timeline.py [fixture] [runs]
"""
from __future__ import annotations

import functools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch

    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.ops import verify as V
    from nodexa_chain_core_amd.parallel import world as W
    from nodexa_chain_core_amd.parallel.verify import verify_headers_distributed

    fixture = sys.argv[1] if len(sys.argv) > 1 else os.path.join("tests", "data", "testnet_mixed_10k.hdr")
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    W.init(use_gpu=True)
    params, headers = synthetic.load(fixture)
    stages: dict[str, float] = {}

    def timed(name, fn):
        @functools.wraps(fn)
        def wrap(*a, **k):
            t = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                stages[name] = stages.get(name, 0.0) + (time.perf_counter() - t) * 1e3
        return wrap

    def timed_run(fn):
        @functools.wraps(fn)
        def wrap(*a, **k):
            t = time.perf_counter()
            finish = fn(*a, **k)
            stages["issue"] = stages.get("issue", 0.0) + (time.perf_counter() - t) * 1e3
            return timed("wait+readback", finish)
        return wrap

    V._grouped = timed("grouped(programs+uploads)", V._grouped)
    V._run_light = timed_run(V._run_light)
    V.gpu_hash_jobs = timed("gpu_hash_jobs", V.gpu_hash_jobs)
    for r in range(runs):
        stages.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = verify_headers_distributed(params, headers, mode="light")
        torch.cuda.synchronize()
        total = (time.perf_counter() - t0) * 1e3
        ok = sum(1 for i in range(len(res)) if res[i]["valid"])
        print(json.dumps({"run": r, "headers": len(headers), "valid": ok, "total_ms": round(total, 3),
                          **{k: round(v, 3) for k, v in stages.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
