#!/usr/bin/env python3
"""Headline benchmark: KawPow MH/s (+ Equihash(200,9) Sol/s), whole node, N MI355X.

BASELINE.json config 2/4: KawPow miner on a synthetic regtest header with a
4 GiB DAG (epoch 384), nonce-range data parallelism over N GPUs (one process
per GPU, RCCL over xGMI): the work packet (header hash, target, height) is
broadcast from rank 0, every rank searches its own disjoint nonce window per
step, and the per-rank share rings are all-gathered on the GPU stream after
every search kernel — the full mining step, nothing skipped.

    python bench.py --gpus N --steps K --warmup W
    (N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
          --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...)

One step = one search window of --batch nonces per GPU (weak scaling).
Timing: W untimed steps, barrier + synchronize, K timed steps, synchronize +
barrier, max elapsed over ranks. Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

def _baseline() -> tuple[float | None, str | None]:
    """The reference publishes no KawPow number. Use a published one if
    BASELINE.json ever gains it, else the reference's own progpow::search measured on
    this container's 8-core host (tools/ref_cpu_baseline.sh -> profiles/ref_cpu_baseline/)."""
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            v = (json.load(f).get("published") or {}).get("kawpow_mhs")
        if v:
            return float(v), "BASELINE.json published.kawpow_mhs"
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(ROOT, "profiles", "ref_cpu_baseline", "epoch384.json")) as f:
            return float(json.load(f)["mhs"]), "reference progpow::search, 8-core host, epoch 384 (BASELINE.md)"
    except (OSError, ValueError, KeyError):
        return None, None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--epoch", type=int, default=384, help="384 -> 4 GiB DAG (BASELINE config)")
    ap.add_argument("--batch", type=int, default=1 << 25,
                    help="nonces per GPU per step (profiles/r2q: 2^25 amortises the kernel tail, +0.9 %% vs 2^23)")
    ap.add_argument("--equihash", type=int, default=12,
                    help="Equihash(200,9): batches of 8 solves per GPU to time (0 = skip)")
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args()

    import torch

    from nodexa_chain_core_amd import _build

    _build.build_all()
    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.chain.header import BlockHeader
    from nodexa_chain_core_amd.ops import jit
    from nodexa_chain_core_amd.ops.ethash import DeviceEpoch
    from nodexa_chain_core_amd.ops.kawpow import KawpowSearcher
    from nodexa_chain_core_amd.parallel import dag as pdag
    from nodexa_chain_core_amd.parallel import world as W
    from nodexa_chain_core_amd.parallel.shares import ShareGather

    world = W.init(use_gpu=True)
    rank, ws = world.rank, world.world_size
    log = (lambda *a: print(*a, file=sys.stderr, flush=True)) if (rank == 0 and not args.quiet) else (lambda *a: None)

    height = args.epoch * _core.EPOCH_LENGTH + 123
    period = height // 3
    # Compile the period kernel before touching the DAG (child-process compile).
    jit.get(period) if rank == 0 else None
    W.barrier()

    # Synthetic regtest header (KawPow layout; time after activation).
    hdr = BlockHeader(version=0x20000000, prev=_core.sha256d(b"nodexa-bench-prev"),
                      merkle_root=_core.sha256d(b"nodexa-bench-merkle"), time=1_700_000_000,
                      bits=0x1b00ffff, height=height)
    work = struct.pack("<32sQII", hdr.progpow_header_hash(), 0, height, 0)
    work = W.broadcast_bytes(work if rank == 0 else None, len(work))
    header_hash, _, height, _ = struct.unpack("<32sQII", work)
    # Target: ~1 share per 2^22 nonces, so the share path is exercised every step.
    target64 = (1 << 64) // (1 << 22)

    t0 = time.time()
    ctx = _core.get_epoch_context(args.epoch)
    log(f"[bench] light cache epoch {args.epoch}: {ctx.light_bytes/2**20:.0f} MiB in {time.time()-t0:.1f}s")
    ep = DeviceEpoch(args.epoch, ctx=ctx, world_size=ws)
    torch.cuda.synchronize()
    t0 = time.time()
    pdag.build_dag(ep)
    torch.cuda.synchronize()
    dag_s = time.time() - t0
    log(f"[bench] DAG {ep.dag_bytes/2**30:.2f} GiB built in {dag_s:.2f}s over {ws} GPU(s)")
    if not ep.l1_matches():
        raise SystemExit("DAG L1 mismatch vs host golden model")

    searcher = KawpowSearcher(ep, height)
    gather = ShareGather(searcher)
    nonce_base = 0x5EED_0000_0000_0000
    batch = args.batch // searcher.block * searcher.block  # whole workgroups of the tuned kernel

    def step(i: int) -> None:
        start = nonce_base + (i * ws + rank) * batch
        searcher.launch(header_hash, start, batch, target64)
        gather.enqueue()

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    W.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
    torch.cuda.synchronize()
    W.barrier()
    elapsed = time.perf_counter() - t_start
    elapsed = W.all_reduce_max(elapsed)

    # Validate the last step's gathered shares bit-exactly on the host.
    shares = gather.collect()
    bad = [s for s in shares if not s.verify_host(height, header_hash)]
    if bad:
        raise SystemExit(f"{len(bad)} invalid shares from the GPU")
    total = batch * ws * args.steps
    mhs = total / elapsed / 1e6

    eq_sols = None
    if args.equihash:
        # Equihash(200,9): every rank solves its own nonces (weak scaling);
        # node Sol/s = all solutions / slowest rank's time.
        from nodexa_chain_core_amd.ops.equihash import EquihashSolver

        solver = EquihashSolver(num_inst=8)
        mk = lambda i, j: hdr.kawpow_input() + struct.pack("<QQQQ", rank, i, j, 0xE9)  # noqa: E731
        solver.solve([mk(-1 & 0xFFFF, j) for j in range(8)])  # warm-up
        torch.cuda.synchronize()
        W.barrier()
        t0 = time.perf_counter()
        found = 0
        # two batches in flight: the GPU solves batch i+1 while the host verifies batch i
        for i in range(args.equihash):
            solver.launch([mk(i, j) for j in range(8)])
            if i >= 1:
                found += sum(len(s) for s in solver.collect())
        found += sum(len(s) for s in solver.collect())
        torch.cuda.synchronize()
        eq_dt = W.all_reduce_max(time.perf_counter() - t0)
        eq_sols = round(W.all_reduce_sum_int(found) / eq_dt, 2)
        del solver
        log(f"[bench] Equihash(200,9): {eq_sols} Sol/s ({args.equihash} x 8 solves per rank)")

    if rank == 0:
        base, base_src = _baseline()
        out = {
            "metric": "KawPow MH/s + Equihash(200,9) Sol/s, whole node at 1/2/4/8 MI355X",
            "value": round(mhs, 3),
            "unit": "MH/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(mhs / base, 3) if base else None,
            "dtype": "u32",
            "data": "synthetic regtest header + sequential nonces; the real epoch DAG generated on the GPU "
                    "(no chain data)",
            "config": {
                "model": f"KawPow (ProgPoW 0.9.4, RAVENCOINKAWPOW) epoch {args.epoch}, "
                         f"{ep.dag_bytes/2**30:.2f} GiB DAG, height {height}",
                "global_batch": batch * ws,
                "seq_len": None,
                "parallelism": f"dp{ws}",
            },
            "shares_last_step": len(shares),
            "dag_build_s": round(dag_s, 3),
            "equihash_sol_per_s": eq_sols,
            "baseline_mhs": base,
            "baseline_source": base_src,
        }
        for k, v in list(out.items()) + [("config." + a, b) for a, b in out["config"].items()]:
            if isinstance(v, (bytes, bytearray)):
                print(f"[bench] warning: field {k} is bytes", file=sys.stderr)
        print(json.dumps(out, default=lambda o: o.hex() if isinstance(o, (bytes, bytearray)) else str(o)), flush=True)
    W.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
