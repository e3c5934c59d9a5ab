"""Category logging with the reference's BCLog names (+ GPU/RCCL/KAWPOW/EQUIHASH).

Parity: BCLog::LogFlags (src/util.h:84-113), LogPrint / LogPrintf,
LogAcceptCategory (src/util.h:116), `-debug=<cat>` / `-debugexclude`,
`debug.log` in the data directory, and the `logging` RPC
(src/rpc/misc.cpp) that toggles categories at run time.
"""
from __future__ import annotations

import os
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
_timestamps = True   # -logtimestamps
_micros = False      # -logtimemicros
log_ips = False      # -logips: peer addresses in net log lines
RECENT_DEBUG_HISTORY_SIZE = 10 * 1_000_000


def timestamp_format(t: float) -> str:
    s = time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(t))
    return s + (".%06dZ" % int(round((t % 1) * 1e6)) if _micros else "Z")


def shrink_debug_file(path: str) -> None:
    """ShrinkDebugFile (src/util.cpp): past 11 MB keep the last 10 MB, cut at a line start."""
    try:
        size = os.path.getsize(path)
    except OSError:
        return
    if size <= RECENT_DEBUG_HISTORY_SIZE * 11 // 10:
        return
    with open(path, "rb") as f:
        f.seek(size - RECENT_DEBUG_HISTORY_SIZE)
        tail = f.read()
    nl = tail.find(b"\n")
    tail = tail[nl + 1:] if 0 <= nl < len(tail) - 1 else tail
    tmp = path + ".shrink"
    with open(tmp, "wb") as f:
        f.write(tail)
    os.replace(tmp, path)


def configure(debug: list[str], exclude: list[str] | None = None, logfile: str | None = None,
              console: bool = True, timestamps: bool = True, micros: bool = False, ips: bool = False,
              shrink: bool | None = None) -> None:
    global _file, _print_to_console, _timestamps, _micros, log_ips
    if logfile and (shrink if shrink is not None else not debug):  # -shrinkdebugfile (default !fDebug)
        shrink_debug_file(logfile)
    with _lock:
        _timestamps, _micros, log_ips = timestamps, micros, ips
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
    line = (timestamp_format(time.time()) + " " if _timestamps else "") + msg.rstrip("\n")
    with _lock:
        if _file is not None:
            _file.write(line + "\n")
        if _print_to_console:
            print(line, file=sys.stderr, flush=True)


def log_print(cat: str, msg: str) -> None:
    if accept(cat):
        log_printf(f"[{cat}] {msg}")
