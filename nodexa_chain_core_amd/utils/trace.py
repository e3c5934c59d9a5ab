"""roctx ranges around the engine's phases ("roctx ranges around template / epoch /
search phases"), so `rocprofv3 --marker-trace` timelines show epoch DAG builds, template
builds, search steps and batch-verify stages next to the kernels.

Uses the rocprofiler-sdk roctx library (what rocprofv3 intercepts); without a profiler
attached the calls are no-ops. NODEXA_ROCTX=0 disables the library load entirely. The reference
has no tracing framework, only -debug=bench timings, which utils/metrics covers.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None


def _load():
    global _lib
    if _lib is None:
        _lib = False
        if os.environ.get("NODEXA_ROCTX", "1") != "0":
            for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    _lib = lib
                    break
                except (OSError, AttributeError):
                    continue
    return _lib


@contextlib.contextmanager
def trace_range(name: str):
    """`with trace_range("dag_build epoch=384"):` — a nested roctx range."""
    lib = _load()
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _load()
    if lib:
        lib.roctxMarkA(name.encode())


def available() -> bool:
    return bool(_load())


def traced(label: str):
    """Decorator form of trace_range for a whole function / method."""
    import functools

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **k):
            lib = _load()
            if not lib:
                return fn(*a, **k)
            lib.roctxRangePushA(label.encode())
            try:
                return fn(*a, **k)
            finally:
                lib.roctxRangePop()
        return wrapper
    return deco
