"""Category logging with the reference's BCLog names (+ GPU/RCCL/KAWPOW/EQUIHASH).

Parity: BCLog::LogFlags (src/util.h:84-113), LogPrint / LogPrintf,
LogAcceptCategory (src/util.h:116), `-debug=<cat>` / `-debugexclude`,
`debug.log` in the data directory, and the `logging` RPC
(src/rpc/misc.cpp) that toggles categories at run time.
"""
from __future__ import annotations

import sys
import threading
import time

CATEGORIES = [
    "net", "tor", "mempool", "http", "bench", "zmq", "db", "rpc", "estimatefee", "addrman", "selectcoins",
    "reindex", "cmpctblock", "rand", "prune", "proxy", "mempoolrej", "libevent", "coindb", "qt", "leveldb",
    "rewards", "assets", "messaging",
    # new (MI355X engine)
    "gpu", "rccl", "kawpow", "equihash", "miner", "validation",
]

_lock = threading.Lock()
_enabled: set[str] = set()
_file = None
_print_to_console = True


def configure(debug: list[str], exclude: list[str] | None = None, logfile: str | None = None,
              console: bool = True) -> None:
    global _file, _print_to_console
    with _lock:
        _enabled.clear()
        if any(d in ("1", "all") for d in debug):
            _enabled.update(CATEGORIES)
        else:
            _enabled.update(d for d in debug if d in CATEGORIES)
        for e in exclude or []:
            _enabled.discard(e)
        if logfile:
            _file = open(logfile, "a", buffering=1)
        _print_to_console = console


def enable(cat: str) -> None:
    with _lock:
        if cat in ("all", "1"):
            _enabled.update(CATEGORIES)
        elif cat in CATEGORIES:
            _enabled.add(cat)


def disable(cat: str) -> None:
    with _lock:
        if cat in ("all", "1"):
            _enabled.clear()
        else:
            _enabled.discard(cat)


def accept(cat: str) -> bool:
    return cat in _enabled


def active() -> dict[str, bool]:
    return {c: c in _enabled for c in CATEGORIES}


def log_printf(msg: str) -> None:
    line = time.strftime("%Y-%m-%dT%H:%M:%SZ ", time.gmtime()) + msg.rstrip("\n")
    with _lock:
        if _file is not None:
            _file.write(line + "\n")
        if _print_to_console:
            print(line, file=sys.stderr, flush=True)


def log_print(cat: str, msg: str) -> None:
    if accept(cat):
        log_printf(f"[{cat}] {msg}")
