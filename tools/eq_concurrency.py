#!/usr/bin/env python3
"""Equihash(200,9) end-to-end Sol/s (wall clock, host verification included, as bench.py times
it) for instances per batch, workgroups per instance and the number of solvers driven round-robin
on separate HIP streams from one process (two ranks sharing one GPU measured 4025 Sol/s against
3657 for one: profiles/r3za_two_rank_rehearsal; 3929 against 3682 in r6u). Solutions are checked
on the device by default, as the mining loop does.

    python tools/eq_concurrency.py --configs 8:32:1 16:32:1 8:32:2
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=["8:32:1", "16:32:1", "8:32:2"],
                    help="inst:groups:solvers")
    ap.add_argument("--solves", type=int, default=192, help="solves per config (per measurement)")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--verify", choices=("device", "host"), default="device",
                    help="device: the eq_verify_slots verdicts (the mining loop's path); host: the C++ "
                         "verifier as well (~225 us per solution on one core: host-bound)")
    a = ap.parse_args()

    import torch

    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    base = bytes(range(108))

    def run(inst, groups, nsolv, tag):
        solvers = [EquihashSolver(num_inst=inst, device=0, groups=groups) for _ in range(nsolv)]
        streams = [torch.cuda.Stream() for _ in range(nsolv)]
        mk = lambda s, i, j: base + struct.pack("<I", (tag << 24) ^ (s << 20) ^ (i << 8) ^ j)  # noqa: E731
        for s, (sv, st) in enumerate(zip(solvers, streams)):  # warm-up
            with torch.cuda.stream(st):
                sv.launch([mk(s, 255, j) for j in range(inst)])
                sv.collect_arrays(verify=a.verify)
        torch.cuda.synchronize()
        batches = max(2, a.solves // (inst * nsolv))
        found = 0
        t0 = time.perf_counter()
        for i in range(batches):
            for s, (sv, st) in enumerate(zip(solvers, streams)):
                with torch.cuda.stream(st):
                    sv.launch([mk(s, i, j) for j in range(inst)])
                if i >= 1:
                    found += sum(len(x) for x in sv.collect_arrays(verify=a.verify))
        for sv in solvers:
            found += sum(len(x) for x in sv.collect_arrays(verify=a.verify))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        solves = batches * inst * nsolv
        fb = sum(sv.fallbacks for sv in solvers)
        fb_log = [x for sv in solvers for x in sv.fallback_log]
        del solvers
        torch.cuda.empty_cache()
        return {"inst": inst, "groups": groups, "solvers": nsolv, "solves": solves, "solutions": found,
                "s": round(dt, 4), "ms_per_solve": round(dt / solves * 1e3, 4), "sol_per_s": round(found / dt, 1),
                "solves_per_s": round(solves / dt, 1), "fallbacks": fb, "fallback_log": fb_log}

    for rep in range(a.reps):
        for k, c in enumerate(a.configs):
            inst, groups, nsolv = (int(x) for x in c.split(":"))
            r = run(inst, groups, nsolv, rep * 16 + k)
            r["rep"] = rep
            print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
