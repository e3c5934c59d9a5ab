#!/usr/bin/env python3
"""Dispatch latency of a one-workgroup kernel on the mining loop's collective stream while two
search windows occupy the GPU.

At N > 1 ranks every MiningService.step launches RCCL kernels (the record all-gather and the work
packet broadcast) on the loop's priority -16 stream (miner/service.py Comm) while the two queued
kawpow_search windows hold every CU slot they can (768-thread workgroups, two per CU). A one-rank
RCCL world runs its collectives as copies (profiles/README r4b), so no ncclKernel has shared the GPU
with the search yet. This probe stands in for it: a 1-workgroup elementwise kernel on a priority -16
stream, launched every `--every-ms` while the windows run, each bracketed by timing events on that
stream; the event span is queue-to-completion of the tiny kernel. The same probe on an idle GPU is
the baseline. Prints one JSON line (p50 / p90 / p99 / max in ms, busy and idle).

    python tools/coll_dispatch_probe.py --epoch 384 --windows 4
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _pct(xs: list[float], q: float) -> float:
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))]


def _probe(torch, stream, x, n: int, every_ms: float, busy=None) -> list[float]:
    """n tiny kernels on `stream`, one every `every_ms` (or until busy() turns false)."""
    pairs = []
    for _ in range(n):
        if busy is not None and not busy():
            break
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            e0.record(stream)
            x.add_(1)  # 64 elements: one workgroup
            e1.record(stream)
        pairs.append((e0, e1))
        time.sleep(every_ms / 1e3)
    stream.synchronize()
    return [a.elapsed_time(b) for a, b in pairs]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--epoch", type=int, default=384)
    ap.add_argument("--windows", type=int, default=4, help="search windows (2^25 nonces) kept queued, two at a time")
    ap.add_argument("--every-ms", type=float, default=2.0)
    ap.add_argument("--idle", type=int, default=200, help="probe launches on the idle GPU (baseline)")
    a = ap.parse_args()

    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.miner.search import GpuSearchDevice, Work

    torch.cuda.set_device(0)
    dev = GpuSearchDevice(0)
    height = a.epoch * _core.EPOCH_LENGTH + 123
    dev.searcher(height)  # DAG + period kernel
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(device=0, priority=-16)  # as miner/service.Comm
    x = torch.zeros(64, dtype=torch.float32, device="cuda:0")
    idle = _probe(torch, stream, x, a.idle, a.every_ms)

    boundary = ((1 << 256) // (1 << 22) - 1).to_bytes(32, "big")
    work = Work(_core.sha256d(b"probe"), boundary, height, 1, 0x9E0_0000_0000, 0)
    count = 1 << 25
    busy_lat: list[float] = []
    t0 = time.perf_counter()
    start = 0
    dev.submit(0, work, start, count)
    dev.submit(1, work, start + count, count)
    start += 2 * count
    slot = 0
    for _ in range(a.windows - 2):
        # probe while this slot's window runs (the other one is queued behind it / beside it)
        ev = dev.events[slot]
        busy_lat += _probe(torch, stream, x, 10_000, a.every_ms, busy=lambda: not ev.query())
        dev.wait(slot)
        dev.submit(slot, work, start, count)
        start += count
        slot ^= 1
    for _ in range(2):
        ev = dev.events[slot]
        busy_lat += _probe(torch, stream, x, 10_000, a.every_ms, busy=lambda: not ev.query())
        dev.wait(slot)
        slot ^= 1
    wall = time.perf_counter() - t0
    dev.close()

    def summary(xs):
        return {"n": len(xs), "p50": round(_pct(xs, 0.5), 4), "p90": round(_pct(xs, 0.9), 4),
                "p99": round(_pct(xs, 0.99), 4), "max": round(max(xs), 4), "mean": round(statistics.mean(xs), 4)}

    print(json.dumps({"probe": "1-workgroup kernel on a priority -16 stream, event span (ms)",
                      "epoch": a.epoch, "windows": a.windows, "search_wall_s": round(wall, 3),
                      "search_mhs": round(a.windows * count / wall / 1e6, 1),
                      "idle": summary(idle), "busy": summary(busy_lat)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
