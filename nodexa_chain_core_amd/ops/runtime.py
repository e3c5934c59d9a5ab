"""Device runtime glue: load the HIP host runtime (`_hip`) and code objects.

`_hip` links libamdhip64.so.7 by SONAME. torch-ROCm ships its own copy of that
library (same SONAME) and must be the one in the process, so torch is imported
*before* `_hip`; `check_single_hip_runtime()` verifies that exactly one HIP
runtime got mapped. All device memory comes from torch tensors and every launch
goes to a torch stream.
"""
from __future__ import annotations

import os
import threading

import torch  # noqa: F401  (must precede _hip: one HIP runtime per process)

from .. import _build

_lock = threading.Lock()
_hip_mod = None
_code_objects: dict[tuple[int, str], object] = {}

KERNEL_DIR = os.path.join(_build.PKG, "kernels")


class NativeUnavailable(RuntimeError):
    """The native HIP path is required but not built/loadable."""


def hip():
    """The `_hip` extension module (raises NativeUnavailable if it is missing)."""
    global _hip_mod
    if _hip_mod is None:
        with _lock:
            if _hip_mod is None:
                try:
                    from .. import _hip as m  # type: ignore[attr-defined]
                except ImportError as e:  # pragma: no cover - exercised on broken installs
                    raise NativeUnavailable(
                        "nodexa _hip extension not built; run `python -m nodexa_chain_core_amd._build`") from e
                _hip_mod = m
                check_single_hip_runtime()
    return _hip_mod


def check_single_hip_runtime() -> None:
    try:
        with open("/proc/self/maps") as f:
            paths = {line.split()[-1] for line in f if "libamdhip64" in line}
    except OSError:
        return
    real = {os.path.realpath(p) for p in paths}
    if len(real) > 1:
        raise RuntimeError(f"two HIP runtimes mapped in one process: {sorted(real)}")


def gpu_available() -> bool:
    return torch.cuda.is_available()


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise NativeUnavailable("no ROCm GPU visible (torch.cuda.is_available() is False)")


def current_stream_handle() -> int:
    return int(torch.cuda.current_stream().cuda_stream)


def load_code_object(path_or_bytes, key: str | None = None):
    """Load a code object on the *current* device (cached per device+key)."""
    h = hip()
    dev = h.get_device()
    if isinstance(path_or_bytes, (bytes, bytearray)):
        img = bytes(path_or_bytes)
        key = key or str(hash(img))
    else:
        key = key or os.path.abspath(path_or_bytes)
        with open(path_or_bytes, "rb") as f:
            img = f.read()
    ck = (dev, key)
    with _lock:
        co = _code_objects.get(ck)
    if co is None:
        co = h.CodeObject(img)
        with _lock:
            _code_objects[ck] = co
    return co


def static_kernel(module: str, name: str):
    """A kernel from one of the static gfx950 code objects built by _build.py."""
    path = os.path.join(KERNEL_DIR, module + ".hsaco")
    if not os.path.exists(path):
        raise NativeUnavailable(f"missing {path}; run `python -m nodexa_chain_core_amd._build kernels`")
    from . import jump_slots

    if module in jump_slots.STAMPED and not jump_slots.stamp_ok(path):
        # computed jumps into a slot table whose layout was not checked: never load it
        raise NativeUnavailable(f"{path} has no valid handler-slot stamp (ops/jump_slots.py); rebuild it with "
                                "`python -m nodexa_chain_core_amd._build kernels`")
    return load_code_object(path).function(name)
