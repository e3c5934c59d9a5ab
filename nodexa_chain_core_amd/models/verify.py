"""Batch header PoW verification (BASELINE config 5).

Reference behaviour: every header arriving in a `headers` message is checked
serially under cs_main by CheckBlockHeader -> GetHashFull (full KawPow in
light mode, ~5 ms of CPU each) (src/validation.cpp:11638-11665, 12017-12035).
Here a batch is verified in bulk:
  * the cheap "mix-only" final hash (keccak-f800 x2) rejects any
    header whose claimed mix_hash does not meet its target before the DAG is
    touched;
  * surviving headers get the full ProgPoW mix recomputed — on the GPU with
    the epoch DAG resident in HBM (ops/verify.py, program interpreted per
    period so one launch covers every period in the batch), or on all host
    cores with the CPU golden model;
  * DarkGravityWave / contextual rules then run on the host header chain.
"""
from __future__ import annotations

import concurrent.futures as cf
import os

from .. import core
from ..chain.header import from_progpow, to_progpow

_core = core()


def _job(params, h):
    """(block_number, header_hash progpow-order, nonce, claimed mix progpow-order, boundary BE)."""
    target, neg, ovf = _core.set_compact(h.bits)
    return (int(h.height), to_progpow(h.kawpow_header_hash()), int(h.nonce64), to_progpow(h.mix_hash),
            target.to_bytes(32, "big") if not (neg or ovf) else bytes(32))


def verify_headers(params, headers, gpus: list[int] | None = None, threads: int = 0,
                   mode: str = "auto") -> list[dict]:
    """Full PoW check of every header: {"valid", "hash", "reason"?} per header.

    gpus: device ids (one host thread per GPU, the batch split in contiguous
    chunks); None/[] = all host cores with the CPU golden model. mode: GPU
    kernel choice, see ops/verify.py."""
    jobs = [_job(params, h) for h in headers]
    out: list[dict] = [{} for _ in jobs]
    todo, eq_todo, legacy = [], [], []
    for i, (bn, hh, nonce, mix, boundary) in enumerate(jobs):
        if headers[i].is_equihash():
            eq_todo.append(i)
            continue
        if headers[i].time < params.kawpow_activation_time:
            legacy.append(i)
            continue
        fin = _core.kawpow_hash_no_verify(bn, hh, mix, nonce)
        if not _core.hash_le(fin, boundary):
            out[i] = {"valid": False, "reason": "high-hash", "hash": _core.u256_hex(from_progpow(fin))}
            continue
        todo.append(i)
    if gpus and todo:
        from ..ops.verify import gpu_full_hash

        def run(dev: int, part: list[int]):
            return part, gpu_full_hash([jobs[i][0] for i in part], [jobs[i][1] for i in part],
                                       [jobs[i][2] for i in part], device=dev, mode=mode)

        k = len(gpus)
        step = -(-len(todo) // k)
        parts = [(d, todo[j * step:(j + 1) * step]) for j, d in enumerate(gpus) if todo[j * step:(j + 1) * step]]
        with cf.ThreadPoolExecutor(max_workers=len(parts)) as ex:
            for part, res in ex.map(lambda a: run(*a), parts):
                for i, (fin, mix) in zip(part, res):
                    out[i] = _finish(jobs[i], fin, mix)
    else:
        threads = threads or (os.cpu_count() or 4)

        def one(i):
            bn, hh, nonce, _, _ = jobs[i]
            ctx = _core.get_epoch_context(bn // _core.EPOCH_LENGTH)
            return _core.kawpow_hash(ctx, bn, hh, nonce)

        with cf.ThreadPoolExecutor(max_workers=threads) as ex:
            for i, (fin, mix) in zip(todo, ex.map(one, todo)):
                out[i] = _finish(jobs[i], fin, mix)
    if eq_todo:
        _verify_equihash(params, headers, eq_todo, out, gpus, threads)
    if legacy:
        _verify_x16r(params, headers, legacy, out, threads)
    return out


def _verify_x16r(params, headers, idxs: list[int], out: list[dict], threads: int) -> None:
    """Pre-KawPow headers: X16R / X16RV2 by nTime (src/primitives/block.cpp:38-55) on the
    host cores (the native hash releases the GIL), then CheckProofOfWork."""
    def one(i):
        h = headers[i]
        fn = _core.x16rv2 if h.time >= params.x16rv2_activation_time else _core.x16r
        return fn(h.legacy80(), h.prev)

    with cf.ThreadPoolExecutor(max_workers=threads or (os.cpu_count() or 4)) as ex:
        for i, hsh in zip(idxs, ex.map(one, idxs)):
            ok = _core.check_proof_of_work(hsh, headers[i].bits, params)
            out[i] = {"valid": bool(ok), "hash": _core.u256_hex(hsh)} if ok else \
                {"valid": False, "reason": "high-hash", "hash": _core.u256_hex(hsh)}


def _verify_equihash(params, headers, idxs: list[int], out: list[dict], gpus, threads: int) -> None:
    """Equihash-extension headers: solution validity (GPU batch kernel when GPUs are given,
    else the C++ verifier on all cores) and SHA256d(header) <= nBits."""
    act = params.kawpow_activation_time
    ok: dict[int, bool]
    if gpus:
        from ..ops.equihash import verify_solutions

        res = verify_solutions([headers[i].equihash_input() for i in idxs], [headers[i].solution for i in idxs],
                               device=gpus[0])
        ok = dict(zip(idxs, res))
    else:
        p = _core.EquihashParams(params.equihash_n, params.equihash_k)

        def one(i):
            h = headers[i]
            if len(h.solution) != p.solution_bytes:
                return False
            return bool(_core.equihash_verify(p, h.equihash_input(), _core.equihash_unpack(p, h.solution))[0])

        with cf.ThreadPoolExecutor(max_workers=threads or (os.cpu_count() or 4)) as ex:
            ok = dict(zip(idxs, ex.map(one, idxs)))
    for i in idxs:
        h = headers[i]
        hsh = h.equihash_hash(act)
        if not ok[i]:
            out[i] = {"valid": False, "reason": "invalid-solution", "hash": _core.u256_hex(hsh)}
        elif not _core.check_proof_of_work(hsh, h.bits, params):
            out[i] = {"valid": False, "reason": "high-hash", "hash": _core.u256_hex(hsh)}
        else:
            out[i] = {"valid": True, "hash": _core.u256_hex(hsh)}


def _finish(job, fin: bytes, mix: bytes) -> dict:
    _, _, _, claimed_mix, boundary = job
    if mix != claimed_mix:
        return {"valid": False, "reason": "invalid-mix-hash", "hash": _core.u256_hex(from_progpow(fin))}
    if not _core.hash_le(fin, boundary):
        return {"valid": False, "reason": "high-hash", "hash": _core.u256_hex(from_progpow(fin))}
    return {"valid": True, "hash": _core.u256_hex(from_progpow(fin))}


def process_headers(chain, headers, adjusted_time: int, gpus: list[int] | None = None, mode: str = "auto") -> dict:
    """ProcessNewBlockHeaders for a batch (src/validation.cpp:12017-12035): PoW of the whole
    batch in bulk (GPU or all cores), then the contextual rules — nBits == DarkGravityWave,
    MTP, future time, version — header by header on the host chain. Like the reference it
    stops at the first invalid header. Returns counts, the first rejection and stage times."""
    import time

    t0 = time.perf_counter()
    pow_res = verify_headers(chain.params, headers, gpus=gpus, mode=mode)
    t1 = time.perf_counter()
    accepted, reject = 0, None
    for i, (h, r) in enumerate(zip(headers, pow_res)):
        if not r["valid"]:
            reject = {"index": i, "reason": r.get("reason", "high-hash")}
            break
        ar = chain.accept_header(h, adjusted_time, False)
        if not ar.ok:
            reject = {"index": i, "reason": ar.reject}
            break
        accepted += 1
    t2 = time.perf_counter()
    return {"accepted": accepted, "reject": reject, "pow_s": t1 - t0, "context_s": t2 - t1}
