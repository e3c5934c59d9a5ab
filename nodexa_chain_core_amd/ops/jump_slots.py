"""Disassembly check of the jump-table op dispatch of kawpow_verify_waves
(hip/kernels/kawpow_verify_light.hip: kwt_table / kwt_op / kwt_merge): in the built gfx950 code,
every one of the 48 handler slots a call can reach must start with its kind's handler and return
with `s_setpc_b64 s[98:99]` inside its 64 bytes, and every call site must be
`s_add_u32 s94 / s_addc_u32 s95 / s_swappc_b64 s[98:99], s[94:95]`. Also checks the inline
per-site tables of the r5o probe variants (tools/verify_waves_variants.hip) when present.
Accepts a code object or a clang offload bundle (hipcc --genco output).

    python -m nodexa_chain_core_amd.ops.jump_slots nodexa_chain_core_amd/kernels/kawpow_verify_light.hsaco

_build.build_kernels runs it on every build of kawpow_verify_light.hsaco and writes a stamp (the
code object's sha256) beside it; runtime.static_kernel refuses to load that code object without a
matching stamp (fail closed: a build that could not run the check yields no verify_waves kernel).
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MATH = ["v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_min_u32", "v_sub_u32", "v_alignbit_b32",
        "v_and_b32", "v_or_b32", "v_xor_b32", "v_ffbh_u32", "v_bcnt_u32_b32"]
MERGE = ["v_lshl_add_u32", "v_xor_b32", "s_sub_u32", "v_alignbit_b32"]
MERGE_INLINE = ["v_lshl_add_u32", "v_xor_b32", "v_alignbit_b32", "v_alignbit_b32"]


def _code_object(path: str, tmp: str) -> str:
    with open(path, "rb") as f:
        if not f.read(24).startswith(b"__CLANG_OFFLOAD_BUNDLE__"):
            return path
    out = os.path.join(tmp, "co.o")
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", "--unbundle", "--input=" + path,
                    "--output=" + out, "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
    return out


STAMPED = {"kawpow_verify_light"}  # code objects that carry a jump-slot stamp


def stamp_path(hsaco: str) -> str:
    return hsaco + ".slots"


def sha256_file(path: str) -> str:
    import hashlib

    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def verify_and_stamp(hsaco: str) -> dict:
    """Check `hsaco`'s handler slots and write its stamp; raise on a bad layout or a missing tool."""
    for tool in ("llvm-objdump", "clang-offload-bundler"):
        if not os.path.exists(os.path.join(LLVM, tool)):
            raise RuntimeError(f"{LLVM}/{tool} missing: cannot check the handler slots of {hsaco}")
    got = check(hsaco)
    if got["n_errors"] or got["tables"] != 1:
        raise RuntimeError(f"kawpow_verify_waves handler slots: {got}")
    with open(stamp_path(hsaco), "w") as f:
        json.dump({"sha256": sha256_file(hsaco), **got}, f)
    return got


def stamp_ok(hsaco: str) -> bool:
    """`hsaco` carries a stamp written by verify_and_stamp for exactly these bytes."""
    try:
        with open(stamp_path(hsaco)) as f:
            st = json.load(f)
        return st.get("sha256") == sha256_file(hsaco) and st.get("n_errors") == 0
    except (OSError, ValueError):
        return False


def check(path: str) -> dict:
    with tempfile.TemporaryDirectory() as tmp:
        obj = _code_object(path, tmp)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", obj],
                             capture_output=True, text=True, check=True).stdout
    ins = []
    for line in dis.splitlines():
        m = re.match(r"\s+(\S+)(.*?)//\s*([0-9A-F]{12}):\s*([0-9A-F ]+)", line)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), m.group(2).strip(), m.group(4).split()))
    at = {a: (op, args) for a, op, args, _ in ins}
    errors = []
    tables = calls = inline_sites = 0

    def slot_ok(base, k, size, want, ret):
        op = at.get(base + k * size, ("", ""))[0]
        if not op.startswith(want):
            errors.append(f"slot {k} at {base + k * size:#x} is {op!r}, want {want}")
        if ret and not any(at.get(base + k * size + o, ("", ""))[0] == "s_setpc_b64" and
                           at[base + k * size + o][1].startswith("s[98:99]") for o in range(0, size, 4)):
            errors.append(f"slot {k} at {base + k * size:#x} has no s_setpc_b64 s[98:99]")

    for i, (a, op, args, enc) in enumerate(ins):
        if op == "s_getpc_b64" and args.startswith("s[94:95]") and i + 1 < len(ins):
            nxt = ins[i + 1]
            if nxt[1] == "s_add_u32" and nxt[2].split(",")[1].strip() == "s94" and len(nxt[3]) == 2:
                tables += 1
                base = a + 4 + int(nxt[3][1], 16)
                if base % 64:
                    errors.append(f"table at {base:#x} not 64-byte aligned")
                for k in range(48):
                    slot_ok(base, k, 64, MATH[k // 4] if k < 44 else MERGE[k - 44], True)
        elif op == "s_getpc_b64" and args.startswith("s[98:99]") and i + 6 < len(ins):
            kind = ins[i + 1][1]
            seq = [x[1] for x in ins[i + 2:i + 7]]
            if kind in ("s_min_u32", "s_and_b32") and seq == ["s_lshl_b32", "s_add_u32", "s_add_u32", "s_addc_u32",
                                                              "s_setpc_b64"]:
                inline_sites += 1
                table, size = (MATH, 32) if kind == "s_min_u32" else (MERGE_INLINE, 16)
                for k, want in enumerate(table):
                    slot_ok(a + 4 + 24, k, size, want, False)
        elif op == "s_swappc_b64":
            calls += 1
            if args.replace(" ", "") != "s[98:99],s[94:95]" or [x[1] for x in ins[i - 2:i]] != ["s_add_u32", "s_addc_u32"]:
                errors.append(f"call at {a:#x}: {op} {args} after {[x[1] for x in ins[i - 2:i]]}")
    return {"tables": tables, "calls": calls, "inline_sites": inline_sites, "errors": errors[:20],
            "n_errors": len(errors)}


if __name__ == "__main__":
    r = check(sys.argv[1])
    print(json.dumps(r))
    sys.exit(1 if r["n_errors"] or not (r["tables"] or r["inline_sites"]) else 0)
