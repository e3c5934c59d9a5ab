"""Resident batch verify of the 10k mixed fixture with the header decode beside the device
(default) and before it (NODEXA_VERIFY_OVERLAP=0), interleaved: wall, host, accept per run."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from nodexa_chain_core_amd import core  # noqa: E402
from nodexa_chain_core_amd.models import synthetic  # noqa: E402
from nodexa_chain_core_amd.models.verify import process_batch_resident  # noqa: E402

_core = core()
FIX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "data", "testnet_mixed_10k.hdr")
params, hs = synthetic.load(FIX)
raw = open(FIX, "rb").read()
act = params.kawpow_activation_time
adj = hs[-1].time + 3600
res = {"1": [], "0": []}
for it in range(13):
    for mode in ("1", "0"):
        os.environ["NODEXA_VERIFY_OVERLAP"] = mode
        chain = _core.HeaderChain(params)
        torch.cuda.synchronize()
        t = time.perf_counter()
        b = _core.HeaderBatch.from_bytes(raw, act)
        r = process_batch_resident(chain, b, adj, device=0)
        dt = (time.perf_counter() - t) * 1e3
        assert r["accepted"] == len(hs), r
        if it:
            res[mode].append({"ms": dt, **{k: r[k] for k in ("host_ms", "accept_ms", "wait_ms", "overlap_ms", "device_ms")}})
for mode, rs in res.items():
    print(json.dumps({"overlap": mode == "1", **{k: round(statistics.median(x[k] for x in rs), 3) for k in rs[0]}}))
