#!/usr/bin/env python3
"""Equihash solver kernels (equihash_ps.hip) with the simple VALU ops in VOP3 form, timed against
the engine's build (the BLAKE2b of eqp_gen is VALU-bound and xor-heavy: 792 of its ~2050 VALU per
digest are VOP2 v_xor_b32). Build on the host, time on the GPU:

  python profiles/r6ac_eq_e64/eq_e64.py build          # -> tools/bin/eqps_{roundtrip,e64}.hsaco
  python profiles/r6ac_eq_e64/eq_e64.py time [windows]  # interleaved, device-verified solutions
"""
from __future__ import annotations

import importlib.util
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
BIN = os.path.join(ROOT, "tools", "bin")


def _rewrite():
    spec = importlib.util.spec_from_file_location("kp_e64", os.path.join(ROOT, "profiles", "r6z_kawpow_e64", "kawpow_e64.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.rewrite


def build() -> None:
    from nodexa_chain_core_amd import _build

    llvm = os.path.join(_build.ROCM, "lib", "llvm", "bin")
    src = os.path.join(_build.HIPDIR, "kernels", "equihash_ps.hip")
    os.makedirs(BIN, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        s = os.path.join(tmp, "k.s")
        subprocess.run([os.path.join(_build.ROCM, "bin", "hipcc"), "-S", "--cuda-device-only", "--offload-arch=" + _build.ARCH,
                        "-O3", "-std=c++17", "-mcode-object-version=5", "-ffp-contract=fast",
                        "-I" + os.path.join(_build.HIPDIR, "kernels"), src, "-o", s], check=True)
        asm = open(s).read()
        e64, counts = _rewrite()(asm)
        print({"rewritten": counts})
        for tag, text in (("roundtrip", asm), ("e64", e64)):
            p = os.path.join(tmp, tag + ".s")
            open(p, "w").write(text)
            o = os.path.join(tmp, tag + ".o")
            subprocess.run([os.path.join(llvm, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                            "-mcpu=" + _build.ARCH, "-mcode-object-version=5", "-c", p, "-o", o], check=True)
            subprocess.run([os.path.join(llvm, "ld.lld"), "-shared", o, "-o", os.path.join(BIN, f"eqps_{tag}.hsaco")],
                           check=True)


def time_objects(windows: int) -> None:
    import torch

    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    objs = {"engine": None, "roundtrip": os.path.join(BIN, "eqps_roundtrip.hsaco"), "e64": os.path.join(BIN, "eqps_e64.hsaco")}
    solvers = {k: EquihashSolver(num_inst=16, device=0, code_object=v) for k, v in objs.items()}
    base = bytes(range(108))
    mk = lambda t, i, j: base + bytes([t, i & 255, (i >> 8) & 255, j])  # noqa: E731
    times = {k: [] for k in objs}
    sols = {k: 0 for k in objs}
    for rnd in range(5):
        for t, (k, sv) in enumerate(solvers.items()):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(windows):
                sv.launch([mk(t, rnd * windows + i, j) for j in range(16)])
                if i >= 1:
                    sols[k] += sum(len(x) for x in sv.collect_arrays(verify="device"))
            sols[k] += sum(len(x) for x in sv.collect_arrays(verify="device"))
            torch.cuda.synchronize()
            times[k].append((time.perf_counter() - t0) / (windows * 16) * 1e3)
    for k in objs:
        print(json.dumps({"object": k, "ms_per_solve_median": round(statistics.median(times[k]), 4),
                          "ms_per_solve": [round(x, 4) for x in times[k]], "solutions": sols[k],
                          "fallbacks": solvers[k].fallbacks}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        time_objects(int(sys.argv[2]) if len(sys.argv) > 2 else 24)
