#!/usr/bin/env python3
"""Per-step host timings of the Equihash mining loop on one GPU (submit, wait, collectives), with
and without a forced one-rank RCCL group (--collectives): where a step's time goes when the
loop's Sol/s drops below the solver's device rate. Prints one JSON line per configuration."""
import argparse
import json
import os
import statistics
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--collectives", action="store_true")
    ap.add_argument("--steps", type=int, default=24)
    a = ap.parse_args()
    import torch

    from nodexa_chain_core_amd import core
    from nodexa_chain_core_amd.miner.equihash_search import EquihashGpuDevice
    from nodexa_chain_core_amd.miner.search import ALGO_EQUIHASH, Work
    from nodexa_chain_core_amd.miner.service import BenchLeader, MiningService
    from nodexa_chain_core_amd.parallel import world as W

    _core = core()
    W.init(use_gpu=True, force_collectives=a.collectives or None)
    prefix = struct.pack("<i32s32sIII", 0x30000000 | _core.EQUIHASH_VERSION_BIT, b"\x11" * 32, b"\x22" * 32,
                         1_700_000_000, 0x1e0fffff, 5)
    work = Work(prefix, ((1 << 252) - 1).to_bytes(32, "big"), 5, 1, 0xE9_0000_0000_0000, 0, ALGO_EQUIHASH)
    dev = EquihashGpuDevice(W.get().device.index, num_inst=16)
    t = {"submit": [], "wait": []}
    sub, wai = dev.submit, dev.wait

    def tsub(*x, **k):
        t0 = time.perf_counter()
        r = sub(*x, **k)
        t["submit"].append((time.perf_counter() - t0) * 1e3)
        return r

    def twait(*x, **k):
        t0 = time.perf_counter()
        r = wai(*x, **k)
        t["wait"].append((time.perf_counter() - t0) * 1e3)
        return r

    dev.submit, dev.wait = tsub, twait
    svc = MiningService(dev, BenchLeader(work), window=16)
    for _ in range(4):
        svc.step()
    torch.cuda.synchronize()
    t["submit"].clear()
    t["wait"].clear()
    steps, colls = [], []
    h0, t0 = svc.hashes_total, time.perf_counter()
    for _ in range(a.steps):
        s0 = time.perf_counter()
        svc.step()
        steps.append((time.perf_counter() - s0) * 1e3)
        colls.append(svc.coll_ms)
    dt = time.perf_counter() - t0
    med = lambda x: round(statistics.median(x), 3)  # noqa: E731
    print(json.dumps({"collectives": a.collectives, "sol_per_s": round((svc.hashes_total - h0) / dt, 1),
                      "step_ms": med(steps), "submit_ms": med(t["submit"]), "wait_ms": med(t["wait"]),
                      "coll_ms": med(colls), "device_ms": round(svc.rank_info()[0]["last_device_ms"], 3)}),
          flush=True)
    svc.leader.shutdown()
    while svc.step():
        pass
    svc.pipe.drain()
    W.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
