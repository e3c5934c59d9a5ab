#!/usr/bin/env python3
"""Headline benchmark: KawPow MH/s (+ Equihash(200,9) Sol/s, + batch header verify), whole node, N MI355X.

BASELINE.json config 2/4: KawPow mining on a synthetic regtest header with a 4 GiB DAG (epoch
384), nonce-range data parallelism over N GPUs, one process per GPU, RCCL over xGMI. The timed
step is the node's own mining loop — `miner/service.MiningService.step`, the code `nodexad
-gpus=...` mines with — driven by a fixed synthetic job (BenchLeader) instead of a chain:

  queue the next 2^25-nonce window on this GPU / take the previous window's shares
  -> all-gather the share records -> all-reduce the hash counters -> rank 0 consumes the shares
  -> broadcast the 96-byte work packet from rank 0.

The DAG is built sharded over the ranks and all-gathered before timing (reported as
dag_build_s). After timing, rank 0 re-hashes up to 8 of the gathered shares with the host
golden model (light mode, `_core.kawpow_hash`) and exits non-zero on any mismatch.

Extras on the same line: Equihash(200,9) Sol/s (config 3) and batch header verification of
the committed 10k-header fixture through models/verify.process_headers, PoW + DGW/contextual,
every header required to be accepted (config 5; per-epoch setup excluded, reported).

    python bench.py --gpus N --steps K --warmup W
    (N>1 either way: bench.py starts its N ranks itself, one child process per GPU, or
     python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
          --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...;
     a WORLD_SIZE that disagrees with --gpus exits 2)

Timing: W untimed steps, barrier + synchronize, K timed steps, synchronize + barrier, max
elapsed over ranks. Rank 0 prints ONE JSON line.
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
VERIFY_FIXTURE = os.path.join(ROOT, "tests", "data", "testnet_mixed_10k.hdr")  # heights 1-10,000 (epochs 0-1)
# heights 2,880,000-2,889,999 (epochs 384-385, 4 GiB DAGs, 64 MiB light caches), on a stored-index anchor
VERIFY_FIXTURE_E384 = os.path.join(ROOT, "tests", "data", "testnet_mixed_e384_10k.hdr")


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
    # a copy of profiles/ref_cpu_baseline/epoch384.json inside the package: profiles/ is not sent
    # to the GPU boxes (.gpurunignore)
    for path in (os.path.join(ROOT, "nodexa_chain_core_amd", "data", "ref_cpu_baseline_epoch384.json"),
                 os.path.join(ROOT, "profiles", "ref_cpu_baseline", "epoch384.json")):
        try:
            with open(path) as f:
                return float(json.load(f)["mhs"]), "reference progpow::search, 8-core host, epoch 384 (BASELINE.md)"
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def _verify_headers_bench(log, fixture: str = VERIFY_FIXTURE) -> dict | None:
    """BASELINE config 5: the 10k-header fixture through ProcessNewBlockHeaders' work — parse the
    wire bytes, PoW of every header, DarkGravityWave + contextual rules, index insert — timed end to
    end (parse included). "resident" is the device-resident pipeline (models/verify.
    process_batch_resident: one upload, PoW + block hashes + DGW nBits on the GPU, one download, the
    serial insert on the host; over N ranks every GPU takes a slice and the results are
    all-gathered over RCCL); "light" is the no-DAG kernel path. Per-epoch setup (DAG, program
    tables) is excluded and reported; the median of 5 timed runs is the number."""
    import functools
    import statistics

    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import process_batch_resident, process_headers
    from nodexa_chain_core_amd.parallel import world as W
    from nodexa_chain_core_amd.parallel.verify import verify_headers_distributed

    if not os.path.exists(fixture):
        return None
    params, headers = synthetic.load(fixture)
    anchor = synthetic.load_anchor(fixture, params)  # the stored index below a fixture past genesis
    new_chain = functools.partial(synthetic.new_chain, params, anchor)
    with open(fixture, "rb") as f:
        raw = f.read()
    act = params.kawpow_activation_time
    adjusted = headers[-1].time + 3600
    n = len(headers)
    w = W.get()
    dev = w.device.index
    epochs = sorted({h.height // _core.EPOCH_LENGTH for h in headers if not h.is_equihash()})
    out = {"headers": n, "fixture": os.path.relpath(fixture, ROOT), "heights": [headers[0].height, headers[-1].height],
           "kawpow_epochs": epochs}

    # a node's header chain exists before a `headers` message arrives: each run gets a fresh
    # chain made (and, after the run, freed) outside the timed region

    def resident(chain):
        t = time.perf_counter()
        b = _core.HeaderBatch.from_bytes(raw, act)  # boundaries + device rows; header objects deferred
        parse = (time.perf_counter() - t) * 1e3
        r = process_batch_resident(chain, b, adjusted, device=dev, world=w)
        r["parse_ms"] = round(parse, 3)
        r["host_ms"] = round(r["host_ms"] + parse, 3)
        r["host_exposed_ms"] = round(r["host_exposed_ms"] + parse, 3)
        return r

    t0 = time.perf_counter()
    warm = resident(new_chain())  # every epoch's DAG and program table
    torch.cuda.synchronize()
    setup = W.all_reduce_max(time.perf_counter() - t0)
    runs = []
    for _ in range(15):  # ~2 ms each: the median of 15 is steady box to box
        chain = new_chain()
        W.barrier()
        t0 = time.perf_counter()
        r = resident(chain)
        # each rank's own time from the common start (a rank that waits for rank 0's verdict or
        # for the all-gather includes that wait), the slowest rank's is the run's
        runs.append((W.all_reduce_max(time.perf_counter() - t0), r))
        if r["accepted"] != n or warm["accepted"] != n:
            raise SystemExit(f"header verify (resident): accepted {r['accepted']}/{n}, first reject {r['reject']}")
    dt = statistics.median(x for x, _ in runs)
    r = min(runs, key=lambda x: abs(x[0] - dt))[1]
    out["resident"] = {"mode": "DAG already resident (mining node)", "headers_per_s": round(n / dt, 1),
                       "ms": round(dt * 1e3, 3),
                       "ms_min_max": [round(min(x for x, _ in runs) * 1e3, 3), round(max(x for x, _ in runs) * 1e3, 3)],
                       "host_ms": r["host_ms"], "host_exposed_ms": r["host_exposed_ms"], "device_ms": r["device_ms"],
                       "parse_ms": r["parse_ms"], "pack_ms": r["pack_ms"],
                       "issue_ms": r["issue_ms"], "overlap_ms": r["overlap_ms"], "wait_ms": r["wait_ms"],
                       "accept_ms": r["accept_ms"],
                       "dgw_on_gpu": r["dgw_gpu"], "parse_included": True,
                       "ranks": "split over the ranks, all-gathered" if r.get("sharded") else
                       ("rank 0, verdict broadcast (batch below NODEXA_VERIFY_SHARD_MIN)" if w.world_size > 1
                        else "one rank"),
                       "first_run_incl_epoch_setup_s": round(setup, 3)}
    log(f"[bench] verify {n} headers at heights {headers[0].height}-{headers[-1].height} (resident): {n / dt:.0f} "
        f"headers/s (host {r['host_ms']:.2f} ms, {r['host_exposed_ms']:.2f} of it beside no device work, device "
        f"{r['device_ms']:.2f} ms, accept {r['accept_ms']:.2f} ms)")
    fn = functools.partial(verify_headers_distributed, mode="light")
    dgw_dev = dev if w.device.type == "cuda" else None
    process_headers(new_chain(), headers, adjusted, verify_fn=fn, dgw_device=dgw_dev)  # light epochs
    torch.cuda.synchronize()
    chain = new_chain()
    W.barrier()
    t0 = time.perf_counter()
    r = process_headers(chain, headers, adjusted, verify_fn=fn, dgw_device=dgw_dev)
    torch.cuda.synchronize()
    W.barrier()
    dt = W.all_reduce_max(time.perf_counter() - t0)
    if r["accepted"] != n:
        raise SystemExit(f"header verify (light): accepted {r['accepted']}/{n}, first reject {r['reject']}")
    out["light"] = {"mode": "light, no DAG (a non-mining node syncing a new epoch)", "headers_per_s": round(n / dt, 1),
                    "ms": round(dt * 1e3, 2), "pow_ms": round(r["pow_s"] * 1e3, 2),
                    "context_ms": round(r["context_s"] * 1e3, 2), "dgw_on_gpu": r["dgw_gpu"]}
    log(f"[bench] verify {n} headers at heights {headers[0].height}-{headers[-1].height} (light, no DAG): "
        f"{n / dt:.0f} headers/s")
    return out


def _equihash_bench(args, hdr, height: int, rank: int, log) -> dict:
    """BASELINE config 3 through the node's mining loop: MiningService.step with an Equihash work
    packet (miner/equihash_search.EquihashGpuDevice: 16 solver instances per window, two windows in
    flight, every solution verified on the device, SHA256d of the candidate headers on the host),
    the same collectives as the KawPow loop. Sol/s = all ranks' distinct valid solutions over the
    slowest rank's time. The standalone solver (two 16-instance launches in flight, device verdicts)
    is timed after it for comparison."""
    import torch

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.miner.equihash_search import EquihashGpuDevice
    from nodexa_chain_core_amd.miner.search import ALGO_EQUIHASH, Work, equihash_block_hash
    from nodexa_chain_core_amd.miner.service import BenchLeader, MiningService
    from nodexa_chain_core_amd.ops.equihash import EquihashSolver
    from nodexa_chain_core_amd.parallel import world as W

    dev_index = W.get().device.index
    prefix = struct.pack("<i32s32sIII", hdr.version | _core.EQUIHASH_VERSION_BIT, hdr.prev, hdr.merkle_root,
                         hdr.time, hdr.bits, height)
    boundary = ((1 << 252) - 1).to_bytes(32, "big")  # ~1 in 16 solutions is a share
    work = Work(prefix, boundary, height, 1, 0xE9_0000_0000_0000, 0, ALGO_EQUIHASH)
    edev = EquihashGpuDevice(dev_index, num_inst=16)
    leader = BenchLeader(work) if rank == 0 else None
    svc = MiningService(edev, leader, window=16)
    svc.step()
    for _ in range(3):
        svc.step()
    torch.cuda.synchronize()
    W.barrier()
    before = svc.hashes_total
    t0 = time.perf_counter()
    for _ in range(args.equihash):
        svc.step()
    edev.synchronize()
    W.barrier()
    dt = W.all_reduce_max(time.perf_counter() - t0)
    sols = svc.hashes_total - before  # all-reduced over the ranks every step
    node_rate = sols / dt
    if leader is not None:
        leader.shutdown()
    while svc.step():
        pass
    svc.pipe.drain()
    bad = checked = 0
    if rank == 0:  # golden verifier + block hash of the shares the loop shipped
        p = _core.EquihashParams(200, 9)
        for s in leader.shares[:4]:
            checked += 1
            ok = _core.equihash_verify(p, prefix + s.nonce256(), _core.equihash_unpack(p, s.solution))[0]
            bad += not (ok and equihash_block_hash(prefix, s.nonce, s.solution) == s.block_hash)
    if W.all_reduce_sum_int(bad):
        raise SystemExit("Equihash shares of the mining loop failed the host check")
    del svc, edev
    # the standalone solver: two launches in flight, every solution checked on the device (as in
    # the loop), at the loop's 16 instances per launch
    solver = EquihashSolver(num_inst=16)
    mk = lambda i, j: prefix + struct.pack("<QQQQ", rank, i, j, 0xE9)  # noqa: E731
    solver.solve([mk(-1 & 0xFFFF, j) for j in range(16)])
    torch.cuda.synchronize()
    W.barrier()
    t0 = time.perf_counter()
    found = 0
    nb = max(1, args.equihash)
    for i in range(nb):
        solver.launch([mk(i, j) for j in range(16)])
        if i >= 1:
            found += sum(len(s) for s in solver.collect_arrays(verify="device"))
    found += sum(len(s) for s in solver.collect_arrays(verify="device"))
    torch.cuda.synchronize()
    sdt = W.all_reduce_max(time.perf_counter() - t0)
    solo = W.all_reduce_sum_int(found) / sdt
    log(f"[bench] Equihash(200,9) node loop: {node_rate:.1f} Sol/s ({args.equihash} steps x 16 solves per rank, "
        f"{sols} solutions in {dt:.3f}s, {checked} shares host-checked); standalone solver {solo:.1f} Sol/s "
        f"({solver.fallbacks} host re-solves)")
    return {"node_sol_per_s": round(node_rate, 2), "standalone_sol_per_s": round(solo, 2),
            "node_vs_standalone": round(node_rate / solo, 4) if solo else None, "steps": args.equihash,
            "solves_per_step": 16, "loop": "miner/service.MiningService.step (Equihash work packet)",
            "shares_checked": checked}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--epoch", type=int, default=384, help="384 -> 4 GiB DAG (BASELINE config)")
    ap.add_argument("--batch", type=int, default=1 << 25,
                    help="nonces per GPU per step (profiles/r2q: 2^25 amortises the kernel tail)")
    ap.add_argument("--equihash", type=int, default=32,
                    help="Equihash(200,9): mining-loop steps (16 solves each) per GPU to time (0 = skip)")
    ap.add_argument("--collectives", action="store_true",
                    help="force the process group even at one rank (one-rank RCCL: every collective of the "
                         "loop, the DAG build and batch verify runs, as on a multi-GPU node)")
    ap.add_argument("--verify", type=int, default=1, help="1: time BASELINE config 5 (batch header verify)")
    ap.add_argument("--check-shares", type=int, default=8, help="shares re-hashed on the host after timing")
    ap.add_argument("--corrupt-dag", action="store_true",
                    help="test hook: damage every 64th DAG item after the build; the share check must fail")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu: rehearse the same loop and collectives on host devices over gloo (tests)")
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args()

    # --gpus N without a launcher: this process becomes rank 0 and starts ranks 1..N-1 itself, as
    # fresh child processes, before anything here touches a GPU (never an exec of this process)
    env_ws = os.environ.get("WORLD_SIZE")
    if env_ws is not None and int(env_ws) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_ws} (launcher and flag disagree)", file=sys.stderr)
        return 2
    if env_ws is None and args.gpus > 1:
        return _run_as_launcher(args)

    import torch

    from nodexa_chain_core_amd import _build

    cpu = args.device == "cpu"
    if cpu:
        _build.build_core()
    else:
        _build.build_all()
    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.chain.header import BlockHeader
    from nodexa_chain_core_amd.miner.search import CpuSearchDevice, Work
    from nodexa_chain_core_amd.miner.service import BenchLeader, MiningService
    from nodexa_chain_core_amd.parallel import world as W

    world = W.init(use_gpu=not cpu, force_collectives=args.collectives or None)
    rank, ws = world.rank, world.world_size
    if os.environ.get("NODEXA_BENCH_FAIL_RANK") == str(rank):  # test hook: one rank dies, the rest must not hang
        raise SystemExit(f"rank {rank}: NODEXA_BENCH_FAIL_RANK")
    log = (lambda *a: print(*a, file=sys.stderr, flush=True)) if (rank == 0 and not args.quiet) else (lambda *a: None)
    sync = (lambda: None) if cpu else torch.cuda.synchronize

    height = args.epoch * _core.EPOCH_LENGTH + 123
    if not cpu:
        from nodexa_chain_core_amd.ops import jit

        # compile this period's kernel (child-process hipcc, cached on disk) before the DAG exists
        jit.get(height // 3) if rank == 0 else None
    W.barrier()

    # synthetic regtest header (KawPow layout); ~1 share per 2^22 nonces so shares flow every step
    hdr = BlockHeader(version=0x20000000, prev=_core.sha256d(b"nodexa-bench-prev"),
                      merkle_root=_core.sha256d(b"nodexa-bench-merkle"), time=1_700_000_000,
                      bits=0x1b00ffff, height=height)
    share_bits = 1 if cpu else 22
    boundary = ((1 << 256) // (1 << share_bits) - 1).to_bytes(32, "big")
    work = Work(hdr.progpow_header_hash(), boundary, height, 1, 0x5EED_0000_0000_0000, 0)

    t0 = time.time()
    ctx = _core.get_epoch_context(args.epoch)
    log(f"[bench] light cache epoch {args.epoch}: {ctx.light_bytes / 2**20:.0f} MiB in {time.time() - t0:.1f}s")
    if cpu:
        dev, block, dag_s = CpuSearchDevice(max_window=args.batch), 1, 0.0
    else:
        from nodexa_chain_core_amd.miner.search import GpuSearchDevice

        dev = GpuSearchDevice(world.device.index, collective_dag=world.collective)
        sync()
        W.barrier()
        t0 = time.time()
        block = dev.searcher(height).block  # sharded DAG build + all-gather, L1 self-check, period kernel
        sync()
        dag_s = W.all_reduce_max(time.time() - t0)
        ep = dev.epochs[args.epoch]
        log(f"[bench] DAG {ep.dag_bytes / 2**30:.2f} GiB built in {dag_s:.2f}s over {ws} GPU(s)")
        if args.corrupt_dag:
            v = ep.dag.view(torch.int32)
            rows = v[:v.numel() // 64 * 64].view(-1, 64)  # one row per 256-byte 2048-bit item
            rows[64::64, :] ^= 0x5A5A5A5A  # the first 64 items are the L1 (checked above); spare them
            sync()
        del ep

    leader = BenchLeader(work) if rank == 0 else None
    svc = MiningService(dev, leader, window=max(block, args.batch // block * block))
    batch = svc.window

    gpu_start = gpu_snapshot(world)  # before the warmup: amdsmi's first call is slow, keep it out of the loop
    svc.step()  # the work packet goes out (the loop starts idle)
    for _ in range(args.warmup):
        svc.step()
    sync()
    W.barrier()
    sync()
    t_start = time.perf_counter()
    ends = []
    for _ in range(args.steps):
        svc.step()
        ends.append(svc.last_end_ms)
    sync()
    W.barrier()
    elapsed = W.all_reduce_max(time.perf_counter() - t_start)
    gpu_end = gpu_snapshot(world)
    total = batch * ws * args.steps
    mhs = total / elapsed / 1e6
    # the same windows on the device clock: window ends 2..K of the timed steps (K - 2 windows; the
    # first interval holds the pipeline's restart from the drained warmup), i.e. the steady-state
    # rate without the host's edges; slowest rank
    dev_span = W.all_reduce_max(max(0.0, (ends[-1] - ends[1]) / 1e3)) if args.steps > 2 else 0.0
    kernel_mhs = batch * ws * (args.steps - 2) / dev_span / 1e6 if dev_span > 0 else None
    # stop every rank's loop (stop packet; the queued window is aborted), then drain
    if leader is not None:
        leader.shutdown()
    while svc.step():
        pass
    svc.pipe.drain()

    checked = bad = 0
    if rank == 0:
        # full host re-hash (light mode) of the gathered shares: mix and final must both match
        t0 = time.time()
        for s in leader.shares[:args.check_shares]:
            checked += 1
            bad += not s.verify_full(height, work.header_hash, work.boundary, ctx=ctx)
        log(f"[bench] {checked} shares re-hashed on the host in {time.time() - t0:.1f}s: {bad} mismatches")
    bad = W.all_reduce_sum_int(bad)
    if args.check_shares and W.all_reduce_sum_int(checked) == 0:
        raise SystemExit("no shares to re-hash: the search produced none")
    if bad:
        raise SystemExit(f"{bad} GPU shares failed the full host re-hash")
    del svc
    dev.close()
    del dev
    if not cpu:
        torch.cuda.empty_cache()

    eq = None
    if args.equihash and not cpu:
        eq = _equihash_bench(args, hdr, height, rank, log)

    verify = _verify_headers_bench(log) if args.verify and not cpu else None
    if verify is not None:
        # the same pipeline at the headline epoch (BASELINE config 5 on a live chain's heights)
        v384 = _verify_headers_bench(log, VERIFY_FIXTURE_E384)
        if v384 is not None:
            verify["resident_e384"], verify["light_e384"] = v384["resident"], v384["light"]
            verify["e384_fixture"] = {k: v384[k] for k in ("fixture", "heights", "kawpow_epochs", "headers")}

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
            "device": args.device,
            "data": "synthetic regtest header + sequential nonces; the real epoch DAG generated on the GPU "
                    "(no chain data)",
            "config": {
                "model": f"KawPow (ProgPoW 0.9.4, RAVENCOINKAWPOW) epoch {args.epoch}, "
                         f"{ep_bytes_gib(args.epoch):.2f} GiB DAG, height {height}",
                "global_batch": batch * ws,
                "seq_len": None,
                "parallelism": f"dp{ws}",
            },
            "loop": "miner/service.MiningService.step (the node's mining loop)",
            "device_clock_mhs": round(kernel_mhs, 3) if kernel_mhs else None,
            # rank 0's GPU at the start / end of the timed KawPow steps (amdsmi; empty when absent)
            "gpu_start": gpu_start,
            "gpu_end": gpu_end,
            "shares_rehashed": checked,
            "dag_build_s": round(dag_s, 3),
            "equihash_sol_per_s": eq["node_sol_per_s"] if eq else None,
            "equihash": eq,
            "verify_headers": verify,
            "verify_headers_per_s": verify["resident"]["headers_per_s"] if verify else None,  # DAG resident (mining node)
            "verify_headers_light_per_s": verify["light"]["headers_per_s"] if verify else None,  # no DAG
            # the same at heights 2,880,000-2,889,999 (epochs 384-385: 4 GiB DAGs, 64 MiB light caches)
            "verify_headers_e384_per_s": verify["resident_e384"]["headers_per_s"] if verify and "resident_e384" in verify
            else None,
            "verify_headers_light_e384_per_s": verify["light_e384"]["headers_per_s"] if verify and "light_e384" in verify
            else None,
            "baseline_mhs": base,
            "baseline_source": base_src,
        }
        print(json.dumps(out), flush=True)
    W.shutdown()
    return 0


def _run_as_launcher(args) -> int:
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: start ranks 1..N-1 as child
    processes of this one (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* in their environment; rank r
    drives GPU r), run rank 0 in a child too, and reap them all. Exit status: the first non-zero
    child status, else 0. Reference analogue: GenerateClores starting its N miner threads itself
    (/root/reference/src/miner.cpp:728-759); here they are processes, one per GPU."""
    import signal
    import socket
    import subprocess
    import threading

    n = args.gpus
    if args.device == "gpu" and os.environ.get("NODEXA_DIST_BACKEND", "nccl") == "nccl":
        import torch  # device_count does not initialise the GPU on this image

        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} but {have} GPU(s) visible; RCCL needs one GPU per rank "
                  "(NODEXA_DIST_BACKEND=gloo lets ranks share a GPU for rehearsals)", file=sys.stderr)
            return 2
    port = os.environ.get("MASTER_PORT")
    if port is None:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = str(s.getsockname()[1])
    procs, pumps = [], []

    def on_term(signum, _frame):  # a launcher told to stop takes its ranks down with it
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, on_term)

    def pump(stream, rank):
        # the one JSON line comes from rank 0's stdout; everything else a rank writes there (gloo's
        # connect notices, native prints) goes to stderr, so stdout carries exactly that line
        for line in iter(stream.readline, b""):
            out = sys.stdout if rank == 0 and line.startswith(b"{") else sys.stderr
            out.buffer.write(line)
            out.flush()

    rc = 0
    term_at = None
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
            p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                 stdout=subprocess.PIPE)
            procs.append(p)
            pumps.append(threading.Thread(target=pump, args=(p.stdout, r), daemon=True))
            pumps[-1].start()
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    # a failed rank leaves the others blocked in a collective: end them now
                    for q in pending:
                        q.send_signal(signal.SIGTERM)
                    term_at = time.monotonic()
            if term_at is not None and time.monotonic() - term_at > 30:
                for q in pending:
                    q.kill()
                term_at = None
            time.sleep(0.05)
    except BaseException:
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise
    for t in pumps:
        t.join(timeout=10)
    return rc


def gpu_snapshot(world) -> dict:
    """Clocks, power and temperature of this rank's GPU (utils/gpuinfo; {} on CPU or without amdsmi)."""
    if world.device.type != "cuda":
        return {}
    from nodexa_chain_core_amd.utils import gpuinfo

    return gpuinfo.snapshot(world.device.index)


def ep_bytes_gib(epoch: int) -> float:
    from nodexa_chain_core_amd import _core

    return _core.full_dataset_num_items(epoch) * 128 / 2**30


if __name__ == "__main__":
    sys.exit(main())
