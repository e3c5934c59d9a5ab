#!/usr/bin/env python3
"""Equihash mining-window probe: the solver at 8 and 16 instances on the node's inputs (80-byte
header prefix || nonce256), per-instance solution counts against the golden solver, host
re-solves (fallbacks) and their stats, and the wall time of each collect. Prints JSON lines."""
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import torch

    from nodexa_chain_core_amd import core
    from nodexa_chain_core_amd.miner.search import equihash_nonce256
    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    _core = core()
    p = _core.EquihashParams(200, 9)
    prefix = struct.pack("<i32s32sIII", 0x30000000 | _core.EQUIHASH_VERSION_BIT, b"\x11" * 32, b"\x22" * 32,
                         1_700_000_000, 0x1e0fffff, 5)
    base = 0xE9_0000_0000_0000
    for ni in (8, 16):
        s = EquihashSolver(num_inst=ni)
        for rep in range(3):
            start = base + rep * ni
            inputs = [prefix + equihash_nonce256(start + k) for k in range(ni)]
            t0 = time.perf_counter()
            s.launch(inputs)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            arrays = s.collect_arrays(verify="device")
            t2 = time.perf_counter()
            rec = {"num_inst": ni, "rep": rep, "launch_sync_ms": round((t1 - t0) * 1e3, 2),
                   "collect_ms": round((t2 - t1) * 1e3, 2), "per_inst": [len(a) for a in arrays],
                   "fallbacks_total": s.fallbacks, "fallback_log": s.fallback_log[-3:]}
            if rep == 0:
                gold = []
                for k in (0, ni // 2 + 1, ni - 1):
                    sols, _ = _core.equihash_solve_cpu(p, inputs[k], 16, 0)
                    g = {tuple(x) for x in sols}
                    d = {tuple(int(v) for v in row) for row in arrays[k]}
                    gold.append({"inst": k, "golden": len(g), "device": len(d), "equal": g == d})
                rec["golden"] = gold
            print(json.dumps(rec), flush=True)
        del s
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
