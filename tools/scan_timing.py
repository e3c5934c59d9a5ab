#!/usr/bin/env python3
"""Time the period-agnostic DAG nonce scanner (ops/verify.DagNonceScanner) per stage."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nodexa_chain_core_amd import _core  # noqa: E402
from nodexa_chain_core_amd.ops import verify  # noqa: E402

sc = verify.DagNonceScanner(0, int(sys.argv[1]) if len(sys.argv) > 1 else 2048)
bound = bytes(32)
hh = _core.sha256d(b"x")
t = time.perf_counter()
sc(100, hh, bound, 0)
torch.cuda.synchronize()
print(f"first call (DAG build etc.) {time.perf_counter() - t:.3f}s", flush=True)
for h in (100, 101, 102, 103, 104, 105):
    t = time.perf_counter()
    sc(h, hh, bound, 5000)
    torch.cuda.synchronize()
    print(f"height {h}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
t = time.perf_counter()
for k in range(20):
    sc(105, hh, bound, k * sc.width)
torch.cuda.synchronize()
print(f"same period x20: {1e3 * (time.perf_counter() - t) / 20:.2f} ms/call", flush=True)
t = time.perf_counter()
_core.kawpow_program_words(40)
print(f"program words: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
