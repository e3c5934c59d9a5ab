#!/usr/bin/env python3
"""BASELINE config 5: batch block-header verification + DarkGravityWave retarget.

Loads a mined synthetic testnet KawPow chain (tests/data/testnet_kawpow_10k.hdr,
models/synthetic.py; built on the GPU when missing) and times
ProcessNewBlockHeaders-style acceptance of the whole batch into a fresh header
chain: full KawPow PoW of every header in bulk (GPU light mode, GPU DAG mode, or
all host cores), then nBits == DGW / MTP / time / version per header.
The reference path (CheckBlockHeader -> GetHashFull, light epoch context, one
header at a time under cs_main) is timed on a sample on one host core.

    python tools/verify_bench.py [--gpus N] [--modes light dag] [--cpu-sample 40]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/verify_bench.py --modes dag
Prints one JSON line per measured path (the torchrun form splits the full-hash work over
ranks and all-gathers the rows over RCCL: parallel/verify.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FIXTURE = os.path.join(ROOT, "tests", "data", "testnet_mixed_10k.hdr")  # 9830 KawPow + 170 Equihash


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--modes", nargs="*", default=["light", "dag", "dag-slab"])
    ap.add_argument("--cpu-sample", type=int, default=40, help="headers timed on the serial reference path")
    ap.add_argument("--cpu-threads", action="store_true", help="also time all-host-core verification of the batch")
    ap.add_argument("--file", default=FIXTURE)
    a = ap.parse_args()

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import LAST_TIMING, process_headers, verify_headers

    if os.path.exists(a.file):
        params, headers = synthetic.load(a.file)
    else:
        t0 = time.time()
        params, headers = synthetic.build_kawpow_chain(
            10000, backend="gpu", progress=lambda i: print(f"[verify_bench] mined {i} headers, {time.time() - t0:.0f}s",
                                                          file=sys.stderr, flush=True))
    adjusted = headers[-1].time + 3600
    n = len(headers)
    bits = {h.bits for h in headers}
    base = {"config": "batch block-verify + DGW (BASELINE config 5)", "headers": n,
            "distinct_nbits": len(bits), "epochs": sorted({h.height // _core.EPOCH_LENGTH for h in headers})}

    # reference path: serial full check per header (CpuPowVerifier == GetHashFull light) + DGW
    chain = _core.HeaderChain(params)
    t = time.perf_counter()
    for h in headers[:a.cpu_sample]:
        r = chain.accept_header(h, adjusted, True)
        assert r.ok, r.reject
    dt = time.perf_counter() - t
    ref = dict(base, path="reference-equivalent serial CPU (1 core, light KawPow + DGW)",
               headers_timed=a.cpu_sample, headers_per_s=round(a.cpu_sample / dt, 2), ms_per_header=round(dt / a.cpu_sample * 1e3, 3))
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(ref), flush=True)

    if a.cpu_threads:
        chain = _core.HeaderChain(params)
        r = process_headers(chain, headers, adjusted, gpus=None)
        tot = r["pow_s"] + r["context_s"]
        print(json.dumps(dict(base, path=f"all host cores ({os.cpu_count()})", accepted=r["accepted"],
                              reject=r["reject"], pow_s=round(r["pow_s"], 3), context_s=round(r["context_s"], 3),
                              headers_per_s=round(n / tot, 1))), flush=True)

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # torchrun: one process per GPU, rows all-gathered over RCCL
        return _distributed(a, params, headers, adjusted, base, ref)

    if a.gpus > 0:
        import torch

        gpus = list(range(min(a.gpus, torch.cuda.device_count())))
        for mode in a.modes:
            # warm-up: code objects plus the per-epoch state of every epoch in the batch (light
            # cache, and the DAG in the dag modes) — once per 7500 blocks on a syncing node,
            # reported separately as epoch_setup_s
            tw = time.perf_counter()
            process_headers(_core.HeaderChain(params), headers[:64], adjusted, gpus=gpus, mode=mode)
            for e in sorted({h.height // _core.EPOCH_LENGTH for h in headers}):
                first = next(h for h in headers if h.height // _core.EPOCH_LENGTH == e)
                verify_headers(params, [first], gpus=gpus, mode=mode)
            eq = [h for h in headers if h.is_equihash()][:1]
            if eq:
                verify_headers(params, eq, gpus=gpus, mode=mode)
            setup = time.perf_counter() - tw
            chain = _core.HeaderChain(params)
            torch.cuda.synchronize()
            r = process_headers(chain, headers, adjusted, gpus=gpus, mode=mode)
            tot = r["pow_s"] + r["context_s"]
            out = dict(base, path=f"GPU {mode} x{len(gpus)}", accepted=r["accepted"], reject=r["reject"],
                       pow_s=round(r["pow_s"], 4), context_s=round(r["context_s"], 4),
                       headers_per_s=round(n / tot, 1), vs_reference_serial=round(n / tot / ref["headers_per_s"], 1),
                       pow_stages_ms={k: round(v * 1e3, 2) for k, v in LAST_TIMING.items()},
                       epoch_setup_s=round(setup, 3))
            print(json.dumps(out), flush=True)
            if r["accepted"] != n:
                return 1
    return 0


def _distributed(a, params, headers, adjusted, base, ref) -> int:
    import functools

    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.models.verify import LAST_TIMING, process_headers
    from nodexa_chain_core_amd.parallel import world as W
    from nodexa_chain_core_amd.parallel.verify import verify_headers_distributed

    w = W.init()
    n = len(headers)
    rc = 0
    for mode in a.modes:
        fn = functools.partial(verify_headers_distributed, mode=mode)
        process_headers(_core.HeaderChain(params), headers, adjusted, verify_fn=fn)  # warm: every epoch + code objects
        W.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = process_headers(_core.HeaderChain(params), headers, adjusted, verify_fn=fn)
        torch.cuda.synchronize()
        W.barrier()
        dt = W.all_reduce_max(time.perf_counter() - t0)
        if w.is_main:
            print(json.dumps(dict(base, path=f"GPU {mode} over {w.world_size} ranks (RCCL all-gather)",
                                  accepted=r["accepted"], reject=r["reject"], pow_s=round(r["pow_s"], 4),
                                  context_s=round(r["context_s"], 4), headers_per_s=round(n / dt, 1),
                                  vs_reference_serial=round(n / dt / ref["headers_per_s"], 1),
                                  pow_stages_ms={k: round(v * 1e3, 2) for k, v in LAST_TIMING.items()})), flush=True)
        rc |= int(r["accepted"] != n)
    W.shutdown()
    return rc


if __name__ == "__main__":
    sys.exit(main())
