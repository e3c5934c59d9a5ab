"""Lock-order checking for the engine's Python-side locks (DEBUG_LOCKORDER equivalent).

Parity: src/sync.cpp:25-183 — with -DDEBUG_LOCKORDER every LOCK() records, per
thread, which locks are already held; the first time lock B is taken while A is
held the pair (A, B) is remembered, and a later acquisition in the opposite
order (B held, then A) is a potential deadlock: the reference prints both
orders and aborts (potential_deadlock_detected, :78).

`make_lock(name)` returns a plain `threading.RLock` normally and a checking
`OrderedLock` when lock-order checking is enabled (`-debuglockorder`, or
NODEXA_DEBUG_LOCKORDER=1 in the environment). Native code is covered by the
ThreadSanitizer build instead (csrc/stress, tests/test_sanitizers.py).
"""
from __future__ import annotations

import os
import threading
import traceback

_enabled = os.environ.get("NODEXA_DEBUG_LOCKORDER", "") not in ("", "0")
_graph_lock = threading.Lock()
_orders: dict[tuple[str, str], str] = {}  # (held, acquired) -> stack where first seen
_held = threading.local()


class PotentialDeadlock(RuntimeError):
    pass


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = bool(on)


def enabled() -> bool:
    return _enabled


def reset() -> None:
    with _graph_lock:
        _orders.clear()


def _stack() -> list[str]:
    s = getattr(_held, "stack", None)
    if s is None:
        s = _held.stack = []
    return s


class OrderedLock:
    """Re-entrant lock that checks the global acquisition order of named locks."""

    def __init__(self, name: str):
        self.name = name
        self._lock = threading.RLock()

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        held = _stack()
        if self.name not in held:
            with _graph_lock:
                for h in held:
                    rev = _orders.get((self.name, h))
                    if rev is not None:
                        raise PotentialDeadlock(
                            f"POTENTIAL DEADLOCK DETECTED: {h} -> {self.name} here, but {self.name} -> {h} "
                            f"was seen before at:\n{rev}")
                    _orders.setdefault((h, self.name), "".join(traceback.format_stack(limit=8)))
        ok = self._lock.acquire(blocking, timeout)
        if ok:
            held.append(self.name)
        return ok

    def release(self) -> None:
        held = _stack()
        for i in range(len(held) - 1, -1, -1):
            if held[i] == self.name:
                del held[i]
                break
        self._lock.release()

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc) -> None:
        self.release()

    # threading.Condition support
    def _is_owned(self) -> bool:
        return self._lock._is_owned()  # type: ignore[attr-defined]

    def _release_save(self):
        held = _stack()
        n = sum(1 for h in held if h == self.name)
        for _ in range(n):
            held.remove(self.name)
        return (self._lock._release_save(), n)  # type: ignore[attr-defined]

    def _acquire_restore(self, state) -> None:
        inner, n = state
        self._lock._acquire_restore(inner)  # type: ignore[attr-defined]
        _stack().extend([self.name] * n)


def make_lock(name: str):
    return OrderedLock(name) if _enabled else threading.RLock()
