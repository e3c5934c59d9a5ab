"""Per-period KawPow kernel compilation (the hipRTC-style JIT of SURVEY §7.3).

A ProgPoW period lasts 3 blocks. For each period the C++ generator
(`_core.kawpow_codegen_hip`, csrc/pow/kawpow_codegen.cpp) emits the period's
straight-line program; it is compiled together with
hip/kernels/kawpow_search.hip into a gfx950 code object by the offline
compiler (`hipcc --genco`, run as a child process — never exec'd in place of
a GPU process). Objects are cached on disk keyed by (period, arch, template
hash), so a restart or the next run of the same height reuses them, and
`prefetch()` compiles the next period on a worker thread while the current one
is mining.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import tempfile
import threading

from .. import _build, _core

TEMPLATE = os.path.join(_build.HIPDIR, "kernels", "kawpow_search.hip")
CACHE_DIR = os.environ.get("NODEXA_KERNEL_CACHE", os.path.join(_build.PKG, "..", ".kernel_cache"))
_pool = cf.ThreadPoolExecutor(max_workers=2, thread_name_prefix="kawpow-jit")
_lock = threading.Lock()
_inflight: dict[tuple, cf.Future] = {}


def _template_digest() -> str:
    h = hashlib.sha256()
    kdir = os.path.join(_build.HIPDIR, "kernels")
    for name in ("kawpow_search.hip", "kernel_params.h", "keccak_device.hpp"):
        with open(os.path.join(kdir, name), "rb") as f:
            h.update(f.read())
    h.update(_build.ARCH.encode())
    return h.hexdigest()[:16]


def _variant_tag(defines: tuple[str, ...]) -> str:
    if not defines:
        return ""
    return "_v" + hashlib.sha256("|".join(sorted(defines)).encode()).hexdigest()[:8]


def object_path(period: int, defines: tuple[str, ...] = ()) -> str:
    # the key covers the template, the generated program text (codegen changes) and the variant
    prog = hashlib.sha256(program_source(period).encode()).hexdigest()[:8]
    return os.path.join(os.path.abspath(CACHE_DIR),
                        f"kawpow_p{period}_{_build.ARCH}_{_template_digest()}{prog}{_variant_tag(defines)}.hsaco")


def program_source(period: int) -> str:
    return _core.kawpow_codegen_hip(period)


def compile_period(period: int, defines: tuple[str, ...] = ()) -> str:
    """Compile (or reuse) the code object for `period`; returns its path.

    `defines` selects tuning variants of the template (e.g. "KP_MIN_WAVES=6")."""
    out = object_path(period, defines)
    if os.path.exists(out):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with tempfile.TemporaryDirectory(prefix="kawpow_jit_") as tmp:
        inc = os.path.join(tmp, f"kawpow_program_p{period}.inc")
        with open(inc, "w") as f:
            f.write(program_source(period))
        tmp_out = os.path.join(tmp, "k.hsaco")
        _build.hipcc_genco(TEMPLATE, tmp_out, defines=[f'KAWPOW_PROGRAM_HEADER="{inc}"', *defines])
        _atomic_copy(tmp_out, out)
    return out


def _atomic_copy(src: str, dst: str) -> None:
    tmp = dst + f".tmp{os.getpid()}"
    with open(src, "rb") as a, open(tmp, "wb") as b:
        b.write(a.read())
    os.replace(tmp, dst)


# Tuned variant of the search template (profiles/README.md has the sweep that
# picked it); NODEXA_KAWPOW_DEFINES="A,B=1" overrides it ("none" = plain template).
# r2l / r2m: digests held in registers (the only digest form since r4b) leave only the 64 KiB L1 table in LDS, so
# two 768-thread workgroups share a CU (6 waves/SIMD instead of 4): +0.7 / +0.8 % in two
# interleaved sweeps; 640 / 896 threads (waves uneven across the 4 SIMDs) and 1024 (64 VGPRs,
# heavy spills) lose.
# r3b / r3c: scheduling fences around each round's cache/math program (KP_SCHED_FENCE) keep the
# DAG merge, and with it the wait for the round's HBM gather, at the end of the round: +3.2 / +3.6 %
# in two interleaved 7-round sweeps (profiles/r3b_r3c_sched_fence).
TUNED_DEFINES: tuple[str, ...] = ("KP_HASHES=1", "KP_DPP", "KP_BARRETT", "KP_SBUFFER", "KP_L1X4", "KP_BLOCK=768",
                                  "KP_MIN_WAVES=6", "KP_NT_DAG", "KP_SCHED_FENCE")
_env = os.environ.get("NODEXA_KAWPOW_DEFINES")
DEFAULT_DEFINES: tuple[str, ...] = TUNED_DEFINES if _env is None else tuple(
    d for d in _env.split(",") if d and d != "none")


def defines_for(dag_bytes: int, defines: tuple[str, ...] | None = None) -> tuple[str, ...]:
    """The variant to compile for a DAG of `dag_bytes`: KP_SBUFFER addresses the DAG with 32-bit
    buffer offsets, so for DAGs of 4 GiB or more (epochs >= 385; measured there: the structured
    form is not bit-exact) it becomes KP_PTR64 (64-bit addresses by one v_mad_u64_u32), at the
    same 768 threads / 6 waves per SIMD: profiles/r6_dag_over_4g, epoch 390, 273.0 MH/s against
    268.6 for the 512-thread pointer form it replaces and 283.3 for the buffer form at epoch 384 on
    the same box (1.2 % of that gap is the larger DAG itself: KP_PTR64 at epoch 384 runs 276.4)."""
    d = DEFAULT_DEFINES if defines is None else tuple(defines)
    if dag_bytes >= 1 << 32 and "KP_SBUFFER" in d:  # 32-bit buffer offsets: 64-bit addresses
        d = tuple("KP_PTR64" if x == "KP_SBUFFER" else x for x in d)
    return d


def prefetch(period: int, defines: tuple[str, ...] | None = None) -> cf.Future:
    """Start compiling `period` in the background (idempotent)."""
    defines = DEFAULT_DEFINES if defines is None else tuple(defines)
    key = (period, defines)
    with _lock:
        fut = _inflight.get(key)
        if fut is None:
            fut = _pool.submit(compile_period, period, defines)
            _inflight[key] = fut
        return fut


def get(period: int, defines: tuple[str, ...] | None = None) -> str:
    return prefetch(period, defines).result()


def hipcc_available() -> bool:
    try:
        subprocess.run([os.path.join(_build.ROCM, "bin", "hipcc"), "--version"], capture_output=True, check=True)
        return True
    except (OSError, subprocess.CalledProcessError):
        return False
