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


def verify_headers(params, headers, gpus: list[int] | None = None, threads: int = 0) -> list[dict]:
    jobs = [_job(params, h) for h in headers]
    out: list[dict] = [{} for _ in jobs]
    todo = []
    for i, (bn, hh, nonce, mix, boundary) in enumerate(jobs):
        if headers[i].time < params.kawpow_activation_time:
            out[i] = {"valid": False, "reason": "pre-kawpow header (X16R) not handled by the batch verifier"}
            continue
        fin = _core.kawpow_hash_no_verify(bn, hh, mix, nonce)
        if not _core.hash_le(fin, boundary):
            out[i] = {"valid": False, "reason": "high-hash", "hash": _core.u256_hex(from_progpow(fin))}
            continue
        todo.append(i)
    if gpus:
        from ..ops.verify import gpu_full_hash

        res = gpu_full_hash([jobs[i][0] for i in todo], [jobs[i][1] for i in todo], [jobs[i][2] for i in todo],
                            device=gpus[0])
        for i, (fin, mix) in zip(todo, res):
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
    return out


def _finish(job, fin: bytes, mix: bytes) -> dict:
    _, _, _, claimed_mix, boundary = job
    if mix != claimed_mix:
        return {"valid": False, "reason": "invalid-mix-hash", "hash": _core.u256_hex(from_progpow(fin))}
    if not _core.hash_le(fin, boundary):
        return {"valid": False, "reason": "high-hash", "hash": _core.u256_hex(from_progpow(fin))}
    return {"valid": True, "hash": _core.u256_hex(from_progpow(fin))}
