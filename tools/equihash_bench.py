#!/usr/bin/env python3
"""Equihash(200,9) GPU solver timing: device-only time per batch (hip events),
solutions per solve and host verification cost, for solver shapes and compile-time variants of
equihash_ps.hip, interleaved in one process.

    python tools/equihash_bench.py --inst 16 --engines ps ps:32 --variants "" EQP_NP=384
    python tools/equihash_bench.py --compile-only --variants EQP_NP=384   # on the build host

Shapes: "ps[:groups[:block[:final_groups]]]". Variants are built to
.kernel_cache/equihash_ps_<tag>.hsaco (hipcc --genco).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def variant_object(defines: tuple[str, ...], source: str = "equihash.hip") -> str | None:
    if not defines:
        return None
    from nodexa_chain_core_amd import _build

    src = os.path.join(_build.HIPDIR, "kernels", source)
    h = hashlib.sha256(("|".join(defines) + source).encode())
    for name in (source, "equihash_device.hpp", "kernel_params.h"):
        with open(os.path.join(_build.HIPDIR, "kernels", name), "rb") as f:
            h.update(f.read())
    out = os.path.join(ROOT, ".kernel_cache", f"{source.split('.')[0]}_{h.hexdigest()[:12]}.hsaco")
    if not os.path.exists(out):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        _build.hipcc_genco(src, out, defines=list(defines))
    return out


SOURCES = {"ps": "equihash_ps.hip"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--inst", type=int, default=8)
    ap.add_argument("--batches", type=int, default=5)
    ap.add_argument("--variants", nargs="*", default=[""])
    ap.add_argument("--compile-only", action="store_true")
    ap.add_argument("--engines", nargs="*", default=["ps"], help="ps[:groups[:block[:final_groups]]]")
    a = ap.parse_args()
    # a variant that starts with "-" (an "-mllvm:..." backend option) is passed with a leading space
    variants = [tuple(x.strip() for x in v.split(",") if x.strip()) for v in a.variants]
    kinds = sorted({e.split(":")[0] for e in a.engines})
    objs = {(k, v): variant_object(v, SOURCES[k]) for k in kinds for v in variants}
    if a.compile_only:
        print(json.dumps({f"{k}:{','.join(v) or 'base'}": o for (k, v), o in objs.items()}))
        return 0
    import torch

    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    cfgs = [(e, v) for e in a.engines for v in variants]

    def make(c):
        f = c[0].split(":")
        g = int(f[1]) if len(f) > 1 and f[1] else None  # None: the solver's own choice (P x instances = 256)
        blk = int(f[2]) if len(f) > 2 else 1024
        fin = int(f[3]) if len(f) > 3 else None
        return EquihashSolver(num_inst=a.inst, device=0, groups=g, block=blk, code_object=objs[(f[0], c[1])],
                              final_groups=fin)

    solvers = {c: make(c) for c in cfgs}
    batches = [[os.urandom(112) for _ in range(a.inst)] for _ in range(a.batches + 1)]
    for s in solvers.values():
        s.solve(batches[0])
    torch.cuda.synchronize()
    res = {c: {"dev_ms": [], "sols": 0, "verify_s": 0.0} for c in cfgs}
    for bt in batches[1:]:
        for c, s in solvers.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.launch(bt)
            e1.record()
            e1.synchronize()
            res[c]["dev_ms"].append(e0.elapsed_time(e1))
            t = time.perf_counter()
            res[c]["sols"] += sum(len(x) for x in s.collect(bt))
            res[c]["verify_s"] += time.perf_counter() - t
    for (e, v), r in res.items():
        per_batch = sum(r["dev_ms"]) / len(r["dev_ms"])
        out = {"engine": e, "variant": ",".join(v) or "base", "inst_per_batch": a.inst,
               "device_ms_per_batch": round(per_batch, 3), "device_ms_per_solve": round(per_batch / a.inst, 3),
               "sols_per_solve": round(r["sols"] / (a.batches * a.inst), 3),
               "device_sol_per_s": round(r["sols"] / (sum(r["dev_ms"]) / 1e3), 1),
               "host_collect_verify_s_per_batch": round(r["verify_s"] / a.batches, 4),
               "fallbacks": solvers[(e, v)].fallbacks, "stats": solvers[(e, v)].stats()}
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
