"""In-tree native build for nodexa_chain_core_amd.

Produces (all inside the package directory, so they travel with a gpurun
snapshot and are what the GPU tests load):

  _core.<abi>.so      CPU consensus/PoW core (g++, pybind11)           csrc/**
  _hip.<abi>.so       HIP host runtime (g++ against torch's libamdhip64) hip/runtime/**
  kernels/*.hsaco     gfx950 code objects for the static kernels      hip/kernels/*.hip
  bin/nodexad         native daemon (JSON-RPC server + miner)          csrc/** + tools

The HIP runtime links the *same* libamdhip64.so that torch ships (no SONAME,
resolved through an rpath into torch/lib): one HIP runtime per process, so
device pointers from torch tensors, torch streams and RCCL communicators are
valid in our kernels. Device code is never linked into the host .so; every
kernel is a code object loaded with hipModuleLoadData, which also serves the
per-period KawPow kernels that are generated at run time (see ops/jit.py).

Usage: python -m nodexa_chain_core_amd._build [--force] [--jobs N] [core|bench|hip|kernels|tsan|asan|fuzz]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import contextlib
import fcntl
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
HIPDIR = os.path.join(PKG, "hip")
BUILD = os.path.join(PKG, "..", "build", "obj")
ARCH = os.environ.get("NODEXA_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-march=x86-64-v3",
            "-fvisibility=hidden"]


def _pybind_includes() -> list[str]:
    import pybind11

    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _torch_lib() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        raise RuntimeError("torch (ROCm build) is required to link the HIP runtime")
    return os.path.join(list(spec.submodule_search_locations)[0], "lib")


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _fresh(target: str, srcs: list[str]) -> bool:
    """`target` exists and is newer than every source and header it is built from: nothing to
    do, whether or not the intermediate objects exist (a gpurun snapshot ships the built .so files
    but not build/)."""
    return os.path.exists(target) and not _newer(target, srcs + _headers(CSRC) + _headers(HIPDIR))


_LOCK_DEPTH = 0


@contextlib.contextmanager
def _build_lock():
    """One build at a time across processes: the ranks of a torchrun job (bench.py builds before
    the process group exists) and pytest workers all call the build; the first one builds, the
    others wait on the lock and then find everything up to date. Re-entrant within a process."""
    global _LOCK_DEPTH
    if _LOCK_DEPTH:
        _LOCK_DEPTH += 1
        try:
            yield
        finally:
            _LOCK_DEPTH -= 1
        return
    d = os.path.join(PKG, "..", "build")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, ".lock"), "a") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        _LOCK_DEPTH = 1
        try:
            yield
        finally:
            _LOCK_DEPTH = 0
            fcntl.flock(f, fcntl.LOCK_UN)


def _link(cmd: list[str], out: str) -> None:
    """Link to a temporary name, then rename over `out`: a process that already mapped the old
    library keeps its inode, and nobody ever opens a half-written one."""
    tmp = f"{out}.tmp{os.getpid()}"
    try:
        _run(cmd + ["-o", tmp])
        os.replace(tmp, out)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def _headers(root: str) -> list[str]:
    return glob.glob(os.path.join(root, "**", "*.h*"), recursive=True)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)


def _compile_all(srcs: list[str], flags: list[str], objdir: str, jobs: int, force: bool,
                 compiler: str = "g++") -> list[str]:
    os.makedirs(objdir, exist_ok=True)
    hdrs = _headers(CSRC) + _headers(HIPDIR)
    todo, objs = [], []
    for s in srcs:
        rel = os.path.relpath(s, PKG).replace(os.sep, "_")
        o = os.path.join(objdir, rel + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            todo.append((s, o))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_run, [compiler, *flags, "-c", s, "-o", o]) for s, o in todo]
        for f in futs:
            f.result()
    return objs


def core_sources() -> list[str]:
    srcs = glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True)
    skip = (os.sep + "daemon" + os.sep, os.sep + "bench" + os.sep, os.sep + "stress" + os.sep, os.sep + "fuzz" + os.sep)
    return sorted(s for s in srcs if not any(k in s for k in skip))


def build_core(force: bool = False, jobs: int = 8) -> str:
    out = os.path.join(PKG, "_core" + EXT)
    with _build_lock():
        if not force and _fresh(out, core_sources()):
            return out
        objs = _compile_all(core_sources(), CXXFLAGS + _pybind_includes(), os.path.join(BUILD, "core"), jobs, force)
        if force or _newer(out, objs):
            _link(["g++", "-shared", *objs, "-pthread"], out)
    return out


def build_bench(force: bool = False, jobs: int = 8) -> str:
    """bin/bench_nodexa: the host micro-benchmarks (csrc/bench) linked with the core objects
    (everything but the pybind11 bindings)."""
    out_dir = os.path.join(PKG, "bin")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "bench_nodexa")
    bench_srcs = sorted(glob.glob(os.path.join(CSRC, "bench", "*.cpp")))
    with _build_lock():
        if not force and _fresh(out, core_sources() + bench_srcs):
            return out
        core_objs = _compile_all(core_sources(), CXXFLAGS + _pybind_includes(), os.path.join(BUILD, "core"), jobs, force)
        core_objs = [o for o in core_objs if "_bind_" not in os.path.basename(o)]
        bench_objs = _compile_all(bench_srcs, CXXFLAGS, os.path.join(BUILD, "bench"), jobs, force)
        objs = core_objs + bench_objs
        if force or _newer(out, objs):
            _link(["g++", *objs, "-pthread"], out)
    return out


SANITIZERS = {"tsan": ["-fsanitize=thread"], "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]}


def build_sanitized(kind: str, force: bool = False, jobs: int = 8) -> str:
    """bin/stress_<kind>: csrc/stress + every core source (no bindings) under ThreadSanitizer
    ("tsan") or AddressSanitizer+UBSan ("asan"); host code only (SURVEY §5 race detection)."""
    san = SANITIZERS[kind]
    flags = ["-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", "-Wall", "-Wno-unused-function", *san]
    srcs = [s for s in core_sources() if os.sep + "bind" + os.sep not in s]
    srcs += sorted(glob.glob(os.path.join(CSRC, "stress", "*.cpp")))
    objs = _compile_all(srcs, flags, os.path.join(BUILD, kind), jobs, force)
    out_dir = os.path.join(PKG, "bin")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "stress_" + kind)
    if force or _newer(out, objs):
        _run(["g++", *san, "-o", out, *objs, "-pthread"])
    return out


def build_fuzz(force: bool = False, jobs: int = 8) -> str:
    """bin/fuzz_nodexa: csrc/fuzz (a libFuzzer entry point) + every core source (no bindings),
    compiled by ROCm's clang with coverage instrumentation and ASan + UBSan, host code only
    (the reference's test_clore_fuzzy tier)."""
    clang = os.path.join(ROCM, "lib", "llvm", "bin", "clang++")
    # nonnull-attribute off: memcpy(dst, nullptr, 0) from empty inputs is defined behaviour from
    # C2y (N3322) and harmless in glibc; every other UB check aborts the run
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-sanitize=nonnull-attribute"]
    # -asan-globals=0: this clang registers some merged string literals twice and aborts with a
    # spurious odr-violation; heap, stack and UB checks are unaffected
    flags = ["-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", "-march=x86-64-v3", "-w",
             "-fsanitize=fuzzer-no-link", "-mllvm", "-asan-globals=0", *san]
    srcs = [s for s in core_sources() if os.sep + "bind" + os.sep not in s]
    srcs += sorted(glob.glob(os.path.join(CSRC, "fuzz", "*.cpp")))
    objs = _compile_all(srcs, flags, os.path.join(BUILD, "fuzz"), jobs, force, compiler=clang)
    out_dir = os.path.join(PKG, "bin")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "fuzz_nodexa")
    if force or _newer(out, objs):
        _run([clang, "-fsanitize=fuzzer", *san, "-o", out, *objs, "-pthread"])
    return out


def build_hip_runtime(force: bool = False, jobs: int = 8) -> str:
    out = os.path.join(PKG, "_hip" + EXT)
    tlib = _torch_lib()
    srcs = sorted(glob.glob(os.path.join(HIPDIR, "runtime", "*.cpp")))
    # The runtime takes host data (light cache, generated program) from _core by
    # pointer/bytes, so it links no core objects: one epoch-context cache per process.
    flags = CXXFLAGS + _pybind_includes() + ["-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROCM, "include")]
    with _build_lock():
        if not force and _fresh(out, srcs):
            return out
        objs = _compile_all(srcs, flags, os.path.join(BUILD, "hip"), jobs, force)
        if force or _newer(out, objs):
            _link(["g++", "-shared", *objs, "-L" + tlib, "-lamdhip64", "-Wl,-rpath," + tlib, "-pthread"], out)
    return out


def hipcc_genco(src: str, out: str, defines: list[str] | None = None, includes: list[str] | None = None) -> None:
    cmd = [os.path.join(ROCM, "bin", "hipcc"), "--genco", "--offload-arch=" + ARCH, "-O3", "-std=c++17",
           "-mcode-object-version=5", "-ffp-contract=fast", "-I" + os.path.join(HIPDIR, "kernels")]
    for d in defines or []:
        if d.startswith("-mllvm:"):  # backend option of a tuning variant, e.g. "-mllvm:-amdgpu-sched-strategy=max-ilp"
            cmd += ["-mllvm", d[len("-mllvm:"):]]
            continue
        if d == "KP_SCHED_ILP":  # tuning variant: the AMDGPU max-ILP machine scheduler
            cmd += ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
        cmd.append("-D" + d)
    for i in includes or []:
        cmd.append("-I" + i)
    _run(cmd + [src, "-o", out])


def build_kernels(force: bool = False, jobs: int = 8) -> list[str]:
    """Static gfx950 code objects (every .hip that is not a per-period template)."""
    kdir = os.path.join(PKG, "kernels")
    os.makedirs(kdir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HIPDIR, "kernels", "*.hip")))
    hdrs = _headers(os.path.join(HIPDIR, "kernels"))
    outs, todo = [], []
    for s in srcs:
        name = os.path.splitext(os.path.basename(s))[0]
        if name.startswith("kawpow_search"):
            continue  # per-period template, compiled by ops/jit.py
        o = os.path.join(kdir, name + ".hsaco")
        outs.append(o)
        if force or _newer(o, [s] + hdrs):
            todo.append((s, o))
    def one(s: str, o: str) -> None:  # compiled under a temporary name, renamed over the old one
        tmp = f"{o}.tmp{os.getpid()}"
        try:
            hipcc_genco(s, tmp)
            os.replace(tmp, o)
        finally:
            if os.path.exists(tmp):
                os.remove(tmp)

    with _build_lock(), cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        todo = [(s, o) for s, o in todo if force or _newer(o, [s] + hdrs)]  # another process may have built them
        for f in [ex.submit(one, s, o) for s, o in todo]:
            f.result()
        # kawpow_verify_waves jumps into handler slots by computed address: stamp the code object
        # only after its slot layout checks out (ops/jump_slots.py); the loader refuses it unstamped
        from .ops import jump_slots

        for o in outs:
            if os.path.splitext(os.path.basename(o))[0] in jump_slots.STAMPED and not jump_slots.stamp_ok(o):
                jump_slots.verify_and_stamp(o)
    return outs


def build_all(force: bool = False, jobs: int = 8, with_hip: bool = True) -> None:
    with _build_lock():
        build_core(force, jobs)
        build_bench(force, jobs)
        if with_hip:
            build_hip_runtime(force, jobs)
            build_kernels(force, jobs)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("what", nargs="*", default=["all"])
    a = ap.parse_args()
    for w in a.what:
        if w in ("all", "core"):
            print(build_core(a.force, a.jobs))
        if w in ("all", "bench"):
            print(build_bench(a.force, a.jobs))
        if w in ("tsan", "asan"):
            print(build_sanitized(w, a.force, a.jobs))
        if w == "fuzz":
            print(build_fuzz(a.force, a.jobs))
        if w in ("all", "hip"):
            print(build_hip_runtime(a.force, a.jobs))
        if w in ("all", "kernels"):
            for k in build_kernels(a.force, a.jobs):
                print(k)


if __name__ == "__main__":
    sys.exit(main())
