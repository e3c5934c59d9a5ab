"""Host-side stages of the resident batch verify on the 10k mixed fixture, each timed alone
(median of 25): wire parse + row pack, native plan, header decode, the index insert's prepare and
commit phases, and the one-phase accept for comparison. CPU only (hashes / nBits from a host chain)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from nodexa_chain_core_amd import core  # noqa: E402
from nodexa_chain_core_amd.models import synthetic  # noqa: E402

_core = core()
FIX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "data", "testnet_mixed_10k.hdr")
params, hs = synthetic.load(FIX)
raw = open(FIX, "rb").read()
act = params.kawpow_activation_time
adj = hs[-1].time + 3600
n = len(hs)
ref = _core.HeaderChain(params)
ref.accept_batch(_core.HeaderBatch.from_bytes(raw, act), adj)
hashes = np.frombuffer(b"".join(ref.at_height(i + 1).hash for i in range(n)), np.uint8).reshape(n, 32).copy()
bits = np.array([h.bits for h in hs], dtype="<u4")
t = {k: [] for k in ("parse", "plan", "decode", "prepare", "commit", "accept_one_phase", "chain_new")}
for it in range(26):
    c0 = time.perf_counter()
    chain = _core.HeaderChain(params)
    c1 = time.perf_counter()
    b = _core.HeaderBatch.from_bytes(raw, act)
    c2 = time.perf_counter()
    b.kawpow_plan(_core.EPOCH_LENGTH)
    c3 = time.perf_counter()
    b.materialize()
    c4 = time.perf_counter()
    p = chain.prepare_batch(b, adj, hashes, bits)
    c5 = time.perf_counter()
    assert chain.commit_batch(p, n) == (n, None, 0)
    c6 = time.perf_counter()
    chain2 = _core.HeaderChain(params)
    b2 = _core.HeaderBatch.from_bytes(raw, act)
    b2.materialize()
    c7 = time.perf_counter()
    assert chain2.accept_batch(b2, adj, hashes, bits, 0, n) == (n, None, 0)
    c8 = time.perf_counter()
    if it:
        for k, v in (("chain_new", c1 - c0), ("parse", c2 - c1), ("plan", c3 - c2), ("decode", c4 - c3),
                     ("prepare", c5 - c4), ("commit", c6 - c5), ("accept_one_phase", c8 - c7)):
            t[k].append(v * 1e3)
print(json.dumps({k: round(statistics.median(v), 3) for k, v in t.items()}))
