#!/usr/bin/env python3
"""KawPow search kernel with its simple VALU ops in the VOP3 (e64) encoding.

profiles/r6y: on gfx950 a stream of v_add / v_sub / v_xor / v_and in the VOP3 encoding issues
~1.55 wave64 instructions per CU per cycle, the same ops in the 32-bit VOP2 encoding 1.03-1.19,
and every other op of the round ~0.90. The compiler picks the short encoding whenever it can. This
tool compiles one period's search kernel to assembly with the production flags, rewrites the
all-VGPR VOP2 forms of those ops to their VOP3 forms (same operation, same operands), assembles and
links the result, and writes:

  <out>/kp_p<period>_roundtrip.hsaco   the unmodified assembly, reassembled (the control)
  <out>/kp_p<period>_e64.hsaco         add/sub/subrev/xor/and/or rewritten

`tools/kawpow_sweep.py --objects name=path ...` times them next to the JIT-built kernel and
re-hashes their shares on the host.

  python profiles/r6z_kawpow_e64/kawpow_e64.py [--period 960041] [--out tools/bin]
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

# VOP2 forms whose operands are all VGPRs: "v_xor_b32_e32 v1, v2, v3"
SIMPLE = re.compile(r"^(\s*)v_(add_u32|sub_u32|subrev_u32|xor_b32|and_b32|or_b32)_e32(\s+)(v\d+), (v\d+), (v\d+)(\s*(;.*)?)$")


def rewrite(asm: str) -> tuple[str, dict[str, int]]:
    counts: dict[str, int] = {}
    out = []
    for line in asm.split("\n"):
        m = SIMPLE.match(line)
        if m:
            counts[m.group(2)] = counts.get(m.group(2), 0) + 1
            line = f"{m.group(1)}v_{m.group(2)}_e64{m.group(3)}{m.group(4)}, {m.group(5)}, {m.group(6)}"
        out.append(line)
    return "\n".join(out), counts


def build(period: int, out_dir: str, defines: tuple[str, ...] | None = None) -> dict[str, str]:
    from nodexa_chain_core_amd import _build
    from nodexa_chain_core_amd.ops import jit

    defines = jit.DEFAULT_DEFINES if defines is None else defines
    llvm = os.path.join(_build.ROCM, "lib", "llvm", "bin")
    os.makedirs(out_dir, exist_ok=True)
    paths = {}
    with tempfile.TemporaryDirectory(prefix="kp_e64_") as tmp:
        inc = os.path.join(tmp, f"kawpow_program_p{period}.inc")
        with open(inc, "w") as f:
            f.write(jit.program_source(period))
        s = os.path.join(tmp, "k.s")
        cmd = [os.path.join(_build.ROCM, "bin", "hipcc"), "-S", "--cuda-device-only", "--offload-arch=" + _build.ARCH,
               "-O3", "-std=c++17", "-mcode-object-version=5", "-ffp-contract=fast",
               "-I" + os.path.join(_build.HIPDIR, "kernels"), f'-DKAWPOW_PROGRAM_HEADER="{inc}"']
        cmd += ["-D" + d for d in defines]
        subprocess.run(cmd + [jit.TEMPLATE, "-o", s], check=True)
        with open(s) as f:
            asm = f.read()
        e64, counts = rewrite(asm)
        print({"period": period, "rewritten": counts}, flush=True)
        for tag, text in (("roundtrip", asm), ("e64", e64)):
            src = os.path.join(tmp, f"{tag}.s")
            with open(src, "w") as f:
                f.write(text)
            obj = os.path.join(tmp, f"{tag}.o")
            subprocess.run([os.path.join(llvm, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                            "-mcpu=" + _build.ARCH, "-mcode-object-version=5", "-c", src, "-o", obj], check=True)
            out = os.path.join(out_dir, f"kp_p{period}_{tag}.hsaco")
            subprocess.run([os.path.join(llvm, "ld.lld"), "-shared", obj, "-o", out], check=True)
            paths[tag] = out
    return paths


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--period", type=int, default=(384 * 7500 + 123) // 3)
    ap.add_argument("--out", default=os.path.join(ROOT, "tools", "bin"))
    a = ap.parse_args()
    for tag, p in build(a.period, a.out).items():
        print(f"{tag}={p}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
