#!/usr/bin/env python3
"""A/B sweep of KawPow search-kernel variants in ONE process (interleaved rounds).

Builds the epoch DAG once, loads every variant's code object, then runs R
rounds x V variants, each a timed search window (hip events), and prints the
median/min MH/s per variant plus a bit-exactness check of one known hash.

    python tools/kawpow_sweep.py --epoch 384 --variants "" "KP_NT_DAG" "KP_MIN_WAVES=6"
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
    ap.add_argument("--batch", type=int, default=1 << 23)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", nargs="*", default=["tuned"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--check-windows", type=int, default=4, help="nonce windows re-hashed per variant")
    ap.add_argument("--raw", action="store_true", help="compile the variants as given (no jit.defines_for)")
    ap.add_argument("--objects", nargs="*", default=[],
                    help="name=path: prebuilt code objects of the same period timed as extra variants "
                         "(e.g. tools/kawpow_e64.py output)")
    a = ap.parse_args()

    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.ops import jit, runtime
    from nodexa_chain_core_amd.ops.ethash import DeviceEpoch

    height = a.epoch * 7500 + 123
    period = height // 3
    # "tuned" = the production variant (ops/jit.py TUNED_DEFINES); "" = the plain template
    # "tuned-X+Y" = the production variant without X and with Y. Every variant goes through
    # jit.defines_for, so at epochs with a DAG of 4 GiB or more the 32-bit buffer forms become
    # pointer loads.
    import re

    def parse(v):
        if v.startswith("tuned"):
            d = list(jit.TUNED_DEFINES)
            for op, x in re.findall(r"([+-])([^+-]+)", v[len("tuned"):]):
                if op == "-":
                    d = [y for y in d if y != x]
                elif x not in d:
                    d.append(x)
            return tuple(d)
        return tuple(x for x in v.split(",") if x)

    dag_bytes = _core.full_dataset_num_items(a.epoch) * 128
    variants = list(dict.fromkeys(parse(v) if a.raw else jit.defines_for(dag_bytes, parse(v)) for v in a.variants))
    paths = {v: jit.get(period, v) for v in variants}
    for spec in a.objects:  # prebuilt objects: keyed ("obj:<name>",)
        name, _, path = spec.partition("=")
        variants.append(("obj:" + name,))
        paths[variants[-1]] = os.path.abspath(path)
    torch.cuda.set_device(0)
    ep = DeviceEpoch(a.epoch, device=0)
    ep.build()
    torch.cuda.synchronize()
    h = runtime.hip()
    res = torch.zeros(h.sizeof_results() // 4, dtype=torch.int32, device="cuda")
    scratch = torch.empty(a.batch * 8, dtype=torch.int32, device="cuda")
    sargs = (scratch.data_ptr(), scratch.numel() * 4)
    kern = {v: runtime.load_code_object(p, key=p).function("kawpow_search") for v, p in paths.items()}
    header = _core.sha256d(b"sweep")
    stream = runtime.current_stream_handle()

    nb = {v: a.batch // k.max_threads * k.max_threads for v, k in kern.items()}  # whole workgroups

    def run(v, start):
        res[:4].zero_()
        h.launch_kawpow_search(kern[v], ep.dag.data_ptr(), ep.items2048, res.data_ptr(), header, start, 0,
                               nb[v], stream, *sargs)

    # bit-exactness: every variant, target = all-pass, EVERY returned share (up to the 64-slot
    # ring) of several nonce windows re-hashed on the CPU golden model
    import struct

    ctx = _core.get_epoch_context(a.epoch)
    hh = bytes(header)
    for v in variants:
        if any(x.startswith("KP_SKEL") for x in v):
            continue  # ceiling skeletons compute something else by construction
        bad = checked = 0
        for w in range(a.check_windows):
            res.zero_()
            h.launch_kawpow_search(kern[v], ep.dag.data_ptr(), ep.items2048, res.data_ptr(), header,
                                   1000 + w * 7919 * 5120, (1 << 64) - 1, -(-5120 // kern[v].max_threads) * kern[v].max_threads,
                                   stream, *sargs)
            raw = res.cpu().numpy().tobytes()
            n = min(struct.unpack_from("<I", raw, 0)[0], 64)
            for i in range(n):
                vals = struct.unpack_from("<Q8I8I", raw, 16 + i * 72)
                fin, mix = _core.kawpow_hash(ctx, height, hh, vals[0])
                ok = struct.pack("<8I", *vals[1:9]) == mix and struct.pack("<8I", *vals[9:17]) == fin
                bad += not ok
                checked += 1
        print(json.dumps({"variant": ",".join(v) or "base", "shares_checked": checked, "mismatches": bad,
                          "bitexact": bad == 0 and checked > 0}), flush=True)
    for v in variants:  # warm
        run(v, 0)
    torch.cuda.synchronize()
    times = {v: [] for v in variants}
    nv = len(variants)
    for r in range(a.rounds):
        # rotate the order every round so position effects (clock drift, L2 state left by the
        # previous variant) are spread evenly over the variants
        for v in variants[r % nv:] + variants[:r % nv]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(v, (r + 1) * a.batch)
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / 1e3)
    rows = []
    for v in variants:
        mhs = [nb[v] / t / 1e6 for t in times[v]]
        rows.append({"variant": ",".join(v) or "base", "median_mhs": round(statistics.median(mhs), 2),
                     "max_mhs": round(max(mhs), 2), "min_mhs": round(min(mhs), 2)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
