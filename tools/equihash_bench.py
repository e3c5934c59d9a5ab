#!/usr/bin/env python3
"""Equihash(200,9) GPU solver timing: device-only time per batch (hip events),
solutions per solve, host verification cost — for several counter-bank
settings, interleaved in one process."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--inst", type=int, default=8)
    ap.add_argument("--batches", type=int, default=5)
    ap.add_argument("--banks", type=int, nargs="*", default=[4])
    a = ap.parse_args()
    import torch

    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    solvers = {b: EquihashSolver(num_inst=a.inst, device=0, banks=b) for b in a.banks}
    batches = [[os.urandom(112) for _ in range(a.inst)] for _ in range(a.batches + 1)]
    for s in solvers.values():
        s.solve(batches[0])
    torch.cuda.synchronize()
    res = {b: {"dev_ms": [], "sols": 0, "verify_s": 0.0} for b in a.banks}
    for bt in batches[1:]:
        for b, s in solvers.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.launch(bt)
            e1.record()
            e1.synchronize()
            res[b]["dev_ms"].append(e0.elapsed_time(e1))
            t = time.perf_counter()
            res[b]["sols"] += sum(len(x) for x in s.collect(bt))
            res[b]["verify_s"] += time.perf_counter() - t
    for b, r in res.items():
        per_batch = sum(r["dev_ms"]) / len(r["dev_ms"])
        out = {"banks": b, "inst_per_batch": a.inst, "device_ms_per_batch": round(per_batch, 3),
               "device_ms_per_solve": round(per_batch / a.inst, 3),
               "sols_per_solve": round(r["sols"] / (a.batches * a.inst), 3),
               "device_sol_per_s": round(r["sols"] / (sum(r["dev_ms"]) / 1e3), 1),
               "host_collect_verify_s_per_batch": round(r["verify_s"] / a.batches, 4),
               "stats": solvers[b].stats()}
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
