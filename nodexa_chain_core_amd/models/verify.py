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
import struct
import time

import numpy as np
from collections.abc import Sequence

from .. import core
from ..utils.trace import traced

_core = core()
LAST_TIMING: dict[str, float] = {}  # stage times of the last verify_headers call


@traced("verify.headers_pow")
def verify_headers(params, headers, gpus: list[int] | None = None, threads: int = 0,
                   mode: str = "auto") -> list[dict]:
    """Full PoW check of every header: {"valid", "hash", "reason"?} per header.

    gpus: device ids (one host thread per GPU, the batch split in contiguous
    chunks); None/[] = all host cores with the CPU golden model. mode: GPU
    kernel choice, see ops/verify.py."""
    act = params.kawpow_activation_time
    hs = [h if isinstance(h, _core.BlockHeader) else _core.BlockHeader.deserialize(h.serialize(act), act)
          for h in headers]
    return _verify_native(params, hs, gpus, threads, mode)


class VerifyResults(Sequence):
    """verify_headers' per-header {"valid", "hash", "reason"?} dicts, built on access: the KawPow
    rows stay as arrays (validity, reason code, 32-byte final hash) so a 10k-header batch costs
    no per-header Python work unless a caller looks at the entries; `first_invalid()` is one
    array scan. Entries of other header kinds (high-hash prefilter, Equihash, X16R) are stored
    as dicts in `extra`."""

    REASONS = ("", "invalid-mix-hash", "high-hash")

    def __init__(self, n: int):
        self.n = n
        self.valid = np.zeros(n, dtype=bool)
        self.code = np.zeros(n, dtype=np.uint8)   # index into REASONS for array-held rows
        self.held = np.zeros(n, dtype=bool)       # row i lives in the arrays
        self.final = np.zeros((n, 32), dtype=np.uint8)
        self.extra: dict[int, dict] = {}
        # block hashes (storage order) the PoW stage produced, for the contextual stage
        self.block_hash = np.zeros((n, 32), dtype=np.uint8)
        self.has_hash = np.zeros(n, dtype=bool)

    def set(self, i: int, d: dict, block_hash: bytes | None = None) -> None:
        self.extra[i] = d
        self.held[i] = False
        self.valid[i] = bool(d.get("valid"))
        if block_hash is not None:
            self.block_hash[i] = np.frombuffer(block_hash, dtype=np.uint8)
            self.has_hash[i] = True

    def hashes_blob(self, upto: int) -> bytes | None:
        """The first `upto` block hashes as one n x 32 blob, or None if any is missing."""
        if upto and self.has_hash[:upto].all():
            return np.ascontiguousarray(self.block_hash[:upto]).tobytes()
        return None

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(self.n))]
        if i < 0:
            i += self.n
        if not 0 <= i < self.n:
            raise IndexError(i)
        if not self.held[i]:
            return self.extra.get(i, {})
        d = {"valid": bool(self.valid[i]), "hash": self.final[i].tobytes().hex()}
        if self.code[i]:
            d["reason"] = self.REASONS[self.code[i]]
        return d

    def first_invalid(self) -> int:
        bad = np.flatnonzero(~self.valid)
        return int(bad[0]) if len(bad) else self.n

    def __eq__(self, other) -> bool:
        return isinstance(other, (list, tuple, VerifyResults)) and list(self) == list(other)

    __hash__ = None


def first_invalid(res) -> int:
    if isinstance(res, VerifyResults):
        return res.first_invalid()
    return next((i for i, r in enumerate(res) if not r["valid"]), len(res))


def _rows_le(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Row-wise big-endian a <= b over (m, 32) uint8 arrays (ethash is_less_or_equal)."""
    diff = a != b
    first = diff.argmax(axis=1)
    r = np.arange(len(a))
    return ~diff.any(axis=1) | (a[r, first] < b[r, first])


def _verify_native(params, headers, gpus, threads: int, mode: str, rows_fn=None) -> list[dict]:
    """verify_headers for C++ BlockHeader batches: job records, boundaries and the
    mix-only prefilter come from one native pass (kawpow_batch_prepare), the GPU result
    rows are checked with numpy, so host time per header stays ~1-2 us."""
    t0 = time.perf_counter()
    n = len(headers)
    if gpus and n >= MIXONLY_GPU_MIN and os.environ.get("NODEXA_MIXONLY", "gpu") == "gpu":
        kinds_b, jobs_b, mix_b, bound_b, pre_b = _prepare_gpu(params, headers, gpus[0])
    else:
        kinds_b, jobs_b, mix_b, bound_b, pre_b = _core.kawpow_batch_prepare(list(headers),
                                                                            params.kawpow_activation_time)
    kinds = np.frombuffer(kinds_b, dtype=np.uint8)
    out = VerifyResults(n)
    pre = np.frombuffer(pre_b, dtype=np.uint8).reshape(n, 32)
    hp = np.flatnonzero(kinds == 1)  # failed the mix-only prefilter: high hash, already final
    out.held[hp], out.code[hp], out.final[hp] = True, 2, pre[hp]
    cand = np.flatnonzero(kinds == 0)
    kp = np.flatnonzero(kinds <= 1)  # KawPow: the mix-only final hash is the block hash (byte-reversed)
    out.block_hash[kp] = pre[kp, ::-1]
    out.has_hash[kp] = True
    t1 = t2 = time.perf_counter()
    if len(cand):
        jobs = np.frombuffer(jobs_b, dtype=np.uint8).reshape(n, 48)[cand]
        if rows_fn is not None:
            res = rows_fn(jobs)
        else:
            res = _gpu_rows(jobs, gpus, mode) if gpus else _cpu_rows(jobs, threads)
        t2 = time.perf_counter()
        mix_ok = (res[:, :32] == np.frombuffer(mix_b, dtype=np.uint8).reshape(n, 32)[cand]).all(axis=1)
        fin = np.ascontiguousarray(res[:, 32:])
        le = _rows_le(fin, np.frombuffer(bound_b, dtype=np.uint8).reshape(n, 32)[cand])
        out.held[cand] = True
        out.final[cand] = fin
        out.valid[cand] = mix_ok & le
        out.code[cand] = np.where(mix_ok, np.where(le, 0, 2), 1)
    t3 = time.perf_counter()
    eq = np.flatnonzero(kinds == 2).tolist()
    if eq:
        _verify_equihash(params, headers, eq, out, gpus, threads)
    t4 = time.perf_counter()
    legacy = np.flatnonzero(kinds == 3).tolist()
    if legacy:
        _verify_x16r(params, headers, legacy, out, threads, gpus)
    LAST_TIMING.update(prepare_s=t1 - t0, kawpow_s=t2 - t1, check_s=t3 - t2, equihash_s=t4 - t3,
                       x16r_s=time.perf_counter() - t4)
    return out


# Batches at least this large take the device prefilter; smaller ones (a block, a few
# headers) stay on the native host pass, whose cost is below a launch's.
MIXONLY_GPU_MIN = 256


def _prepare_gpu(params, headers, device: int):
    """kawpow_batch_prepare's outputs with the mix-only stage on the GPU: the host only sorts the
    header kinds and lays out the 120-byte KawPow headers (_core.kawpow_batch_headers)."""
    from ..ops.sha256 import kawpow_mixonly_batch

    n = len(headers)
    kinds_b, raw_b = _core.kawpow_batch_headers(list(headers), params.kawpow_activation_time)
    kinds = np.frombuffer(kinds_b, dtype=np.uint8).copy()
    raw = np.frombuffer(raw_b, dtype=np.uint8).reshape(n, 120)
    kp = np.flatnonzero(kinds == 0)
    rows = np.zeros((n, 128), np.uint8)
    rows[kp] = kawpow_mixonly_batch(raw[kp], device)
    pre, bound = rows[:, 32:64], rows[:, 64:96]
    kinds[kp[~_rows_le(np.ascontiguousarray(pre[kp]), np.ascontiguousarray(bound[kp]))]] = 1
    jobs = np.zeros((n, 48), np.uint8)
    jobs[:, :32] = rows[:, :32]
    jobs[:, 32:40] = raw[:, 80:88]   # nNonce64 (LE)
    jobs[:, 40:44] = raw[:, 76:80]   # nHeight (LE)
    return (kinds.tobytes(), jobs.tobytes(), np.ascontiguousarray(rows[:, 96:128]).tobytes(),
            np.ascontiguousarray(bound).tobytes(), np.ascontiguousarray(pre).tobytes())


def _gpu_rows(jobs: np.ndarray, gpus: list[int], mode: str) -> np.ndarray:
    """(m, 64) mix||final rows, the batch split in contiguous chunks, one host thread per GPU."""
    from ..ops.verify import gpu_hash_jobs

    if len(gpus) == 1:
        return gpu_hash_jobs(jobs, device=gpus[0], mode=mode)
    chunks = [c for c in np.array_split(np.arange(len(jobs)), len(gpus)) if len(c)]
    with cf.ThreadPoolExecutor(max_workers=len(chunks)) as ex:
        parts = list(ex.map(lambda a: gpu_hash_jobs(jobs[a[1]], device=a[0], mode=mode), zip(gpus, chunks)))
    return np.concatenate(parts)


def _cpu_rows(jobs: np.ndarray, threads: int) -> np.ndarray:
    """Same rows from the C++ golden model (light epoch contexts) on all host cores."""
    def one(k):
        j = jobs[k]
        bn = int.from_bytes(j[40:44].tobytes(), "little")
        ctx = _core.get_epoch_context(bn // _core.EPOCH_LENGTH)
        fin, mix = _core.kawpow_hash(ctx, bn, j[:32].tobytes(), int.from_bytes(j[32:40].tobytes(), "little"))
        return mix + fin

    with cf.ThreadPoolExecutor(max_workers=threads or (os.cpu_count() or 4)) as ex:
        rows = list(ex.map(one, range(len(jobs))))
    return np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(len(jobs), 64)


# Legacy-header batches at least this large hash on the GPU (hip/kernels/x16r.hip: 16 rounds of
# slot-grouped launches, ~1.7 M hashes/s on 65k headers); smaller ones stay on the host cores.
X16R_GPU_MIN = 512


def x16r_hashes(params, legacy80: list[bytes], times: list[int], gpu: int | None) -> list[bytes]:
    """X16R / X16RV2 (by nTime, src/primitives/block.cpp:38-55) hashes of legacy headers: one
    batch on `gpu` (ops/x16r) when it is large enough, else the native host hash on all cores
    (it releases the GIL)."""
    v2 = [t >= params.x16rv2_activation_time for t in times]
    if gpu is not None and len(legacy80) >= X16R_GPU_MIN:
        from ..ops.x16r import x16r_hash_batch

        got = x16r_hash_batch(b"".join(legacy80), v2=np.array(v2), device=gpu)
        return [bytes(r) for r in got]

    def one(k):
        fn = _core.x16rv2 if v2[k] else _core.x16r
        return fn(legacy80[k], legacy80[k][4:36])

    with cf.ThreadPoolExecutor(max_workers=os.cpu_count() or 4) as ex:
        return list(ex.map(one, range(len(legacy80))))


def _verify_x16r(params, headers, idxs: list[int], out: list[dict], threads: int, gpus=None) -> None:
    """Pre-KawPow headers: X16R / X16RV2 (x16r_hashes), then CheckProofOfWork."""
    hs = x16r_hashes(params, [headers[i].legacy80() for i in idxs], [headers[i].time for i in idxs],
                     gpus[0] if gpus else None)
    for i, hsh in zip(idxs, hs):
        ok = _core.check_proof_of_work(hsh, headers[i].bits, params)
        out.set(i, {"valid": bool(ok), "hash": _core.u256_hex(hsh)} if ok else
                {"valid": False, "reason": "high-hash", "hash": _core.u256_hex(hsh)}, hsh)


def _verify_equihash(params, headers, idxs: list[int], out: list[dict], gpus, threads: int) -> None:
    """Equihash-extension headers: solution validity and SHA256d(header) <= nBits — on the GPU
    (eq_verify + sha256d_batch) when GPUs are given, else the C++ verifier on all cores."""
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
    hashes = {}
    if gpus:  # block hash = SHA256d(serialized header) on the device (ops/sha256.py)
        from ..ops.sha256 import sha256d_batch

        ser = [headers[i].serialize(act) for i in idxs]
        if len({len(x) for x in ser}) == 1:
            hashes = dict(zip(idxs, (r.tobytes() for r in sha256d_batch(ser, device=gpus[0]))))
    for i in idxs:
        h = headers[i]
        hsh = hashes.get(i) or h.equihash_hash(act)
        if not ok[i]:
            out.set(i, {"valid": False, "reason": "invalid-solution", "hash": _core.u256_hex(hsh)}, hsh)
        elif not _core.check_proof_of_work(hsh, h.bits, params):
            out.set(i, {"valid": False, "reason": "high-hash", "hash": _core.u256_hex(hsh)}, hsh)
        else:
            out.set(i, {"valid": True, "hash": _core.u256_hex(hsh)}, hsh)


DGW_GPU_MIN = 256  # batches from this size get their DGW nBits from the GPU kernel


@traced("verify.process_headers")
def process_headers(chain, headers, adjusted_time: int, gpus: list[int] | None = None, mode: str = "auto",
                    verify_fn=None, dgw_device: int | None = None) -> dict:
    """ProcessNewBlockHeaders for a batch (src/validation.cpp:12017-12035): PoW of the whole
    batch in bulk (GPU or all cores), then the contextual rules — nBits == DarkGravityWave,
    MTP, future time, version — header by header on the host chain. Like the reference it
    stops at the first invalid header. Returns counts, the first rejection and stage times.
    verify_fn(params, headers) replaces the PoW stage (parallel/verify.py: across ranks).
    dgw_device (default: the first of `gpus`): the GPU that computes every header's
    DarkGravityWave nBits in one launch for batches of DGW_GPU_MIN or more (ops/dgw.py); the
    host stage then only checks them and updates the index."""

    t0 = time.perf_counter()
    pow_res = verify_fn(chain.params, headers) if verify_fn is not None else \
        verify_headers(chain.params, headers, gpus=gpus, mode=mode)
    t1 = time.perf_counter()
    first_bad = first_invalid(pow_res)
    accepted, reject = 0, None
    # contextual checks of the PoW-valid prefix in one native call (GIL released), with the block
    # hashes the PoW stage already computed
    known = pow_res.hashes_blob(first_bad) if isinstance(pow_res, VerifyResults) else None
    prefix = list(headers[:first_bad])
    if dgw_device is None and gpus:
        dgw_device = gpus[0]
    bits = None
    if dgw_device is not None and known is not None and first_bad >= DGW_GPU_MIN:
        from ..ops import dgw  # every header's DarkGravityWave nBits in one launch (hip/kernels/dgw.hip)

        bits = dgw.batch_bits(chain, prefix, known, dgw_device)
    t_dgw = time.perf_counter()
    accepted, why, _ = chain.accept_headers_summary(prefix, adjusted_time, False, known, bits)
    if why is not None:
        reject = {"index": accepted, "reason": why}
    if reject is None and first_bad < len(headers):
        reject = {"index": first_bad, "reason": pow_res[first_bad].get("reason", "high-hash")}
    t2 = time.perf_counter()
    return {"accepted": accepted, "reject": reject, "pow_s": t1 - t0, "context_s": t2 - t1,
            "dgw_gpu": bits is not None, "dgw_s": t_dgw - t1}


_RESIDENT: dict[int, object] = {}


def resident_verifier(device: int):
    from ..ops.header_batch import ResidentHeaderVerifier

    v = _RESIDENT.get(device)
    if v is None:
        v = _RESIDENT[device] = ResidentHeaderVerifier(device)
    return v


@traced("verify.process_batch_resident")
def resident_ready(headers, act: int, device: int, mode: str = "auto") -> bool:
    """Whether a header batch should take the device-resident path (process_batch_resident): always
    for mode "dag"; for "auto" when every epoch of its KawPow headers already has a resident DAG on
    `device` or has more headers than ops/verify.LIGHT_MAX_JOBS (the DAG build then pays for
    itself); "light" never (no DAG is built for a P2P `headers` message of 2000 headers)."""
    if mode == "dag":
        return True
    if mode != "auto":
        return False
    from ..ops import verify as V

    epochs: dict[int, int] = {}
    for h in headers:
        if h.time >= act and not h.is_equihash():
            e = int(h.height) // _core.EPOCH_LENGTH
            epochs[e] = epochs.get(e, 0) + 1
    return bool(epochs) and all(V.is_resident(device, e) or n > V.LIGHT_MAX_JOBS for e, n in epochs.items())


def shard_min_headers() -> int:
    """Smallest batch the resident verify splits over the ranks of a world (NODEXA_VERIFY_SHARD_MIN,
    default 65536). Below it one rank verifies the whole batch and broadcasts the verdict: a 10k
    batch costs ~1.4 ms on one MI355X, of which ~0.6 ms is device work already hidden under the host
    decode + prepare (both spread over the host cores by parallel_for inside the one rank), so a
    split saves no critical-path time and adds an all-gather (profiles/README r6: 2 ranks sharing a
    GPU measured 3.0 M headers/s sharded against 7.4 M on one rank)."""
    return int(os.environ.get("NODEXA_VERIFY_SHARD_MIN", "65536"))


_VERDICT = 96  # broadcast packet: accepted u32 | reject index i32 | dos i32 | reason (84 bytes, utf-8)


def _broadcast_verdict(world, r: dict | None) -> dict | None:
    """Rank 0's verdict to every rank of `world` (one 96-byte broadcast): the others' result dict
    carries the same accepted count and reject, and no timings of their own."""
    from ..parallel import world as W

    pkt = None
    if world.rank == 0 and isinstance(r, BaseException):  # rank 0 failed: every rank raises
        pkt = struct.pack("<Iii84s", 0xFFFFFFFE, -1, 0, repr(r).encode()[:84])
    elif world.rank == 0 and r is None:  # rank 0 could not take the batch: every rank falls back
        pkt = struct.pack("<Iii84s", 0xFFFFFFFF, -1, 0, b"")
    elif world.rank == 0:
        rej = r["reject"] or {}
        why = (rej.get("reason") or "").encode()[:84]
        pkt = struct.pack("<Iii84s", r["accepted"], rej.get("index", -1) if rej else -1, r.get("dos", 0), why)
    raw = W.broadcast_bytes(pkt, _VERDICT)
    if world.rank == 0:
        if isinstance(r, BaseException):
            raise r
        return r
    acc, idx, dos, why = struct.unpack("<Iii84s", raw)
    if acc == 0xFFFFFFFF:
        return None
    if acc == 0xFFFFFFFE:
        raise RuntimeError("batch verify failed on rank 0: " + why.rstrip(b"\0").decode(errors="replace"))
    why = why.rstrip(b"\0").decode()
    return {"accepted": acc, "reject": {"index": idx, "reason": why} if idx >= 0 else None, "dos": dos,
            "pow_s": 0.0, "context_s": 0.0, "dgw_gpu": True, "resident": True, "sharded": False,
            "host_ms": 0.0, "host_exposed_ms": 0.0, "overlap_ms": 0.0, "device_ms": 0.0, "pack_ms": 0.0,
            "issue_ms": 0.0, "wait_ms": 0.0, "accept_ms": 0.0}


def process_batch_resident(chain, batch, adjusted_time: int, device: int = 0, world=None) -> dict | None:
    """ProcessNewBlockHeaders for a native HeaderBatch with the device-resident pipeline
    (ops/header_batch.py): one upload, PoW + block hashes + DGW nBits of every header on the GPU,
    one download, then the serial index insert on the host (HeaderChain.accept_batch). Pre-KawPow
    (X16R) headers, if any, are hashed on the host cores. Same result as process_headers; None when
    the batch does not suit the resident path (not in height order), so the caller falls back.

    Over a world of N ranks (every rank calls with the same batch): a batch of shard_min_headers()
    or more has its device work split in contiguous slices and the codes + block hashes all-gathered;
    a smaller one is verified whole by rank 0 (which commits it to its chain) and the verdict is
    broadcast, so N GPUs never verify slower than one plus a 96-byte broadcast."""
    if world is not None and world.collective and world.world_size > 1 and len(batch) < shard_min_headers():
        r = None
        if world.rank == 0:
            try:
                r = process_batch_resident(chain, batch, adjusted_time, device, None)
            except Exception as e:  # noqa: BLE001 - the other ranks wait in the broadcast: tell them
                r = e
        return _broadcast_verdict(world, r)
    from ..ops.header_batch import CODES

    t0 = time.perf_counter()
    # a peer-chosen batch the resident path cannot take whole goes to process_headers, which
    # rejects the bad header with its DoS score and keeps the valid prefix: an Equihash header whose
    # solution is not 1344 bytes, or more KawPow epochs than the resident-DAG LRU holds (a DAG an
    # in-flight range still reads must not be evicted by the next range's build)
    if len(batch) == 0 or not batch.eq_uniform:
        return None
    from ..ops import verify as V

    v = resident_verifier(device)
    plan = v.plan(batch)
    if plan is None or len({r[0] for r in plan["ranges"]}) > V.MAX_RESIDENT_DAGS:
        return None
    params = chain.params
    series = chain.dgw_ancestors(batch.header(0).prev)
    # while the device verifies, the host decodes the header objects the index insert needs
    # (HeaderBatch.from_bytes defers them) and, once the block hashes and DGW nBits are back (they
    # come before the full hashes), runs the insert's read-only prepare phase; the commit of the
    # verified prefix follows the verdicts. NODEXA_VERIFY_OVERLAP=0: decode first, no prepare.
    overlap_on = os.environ.get("NODEXA_VERIFY_OVERLAP", "1") != "0"
    if not overlap_on:
        batch.materialize()
    prepared = []
    no_legacy = not bool((plan["kinds"] == 3).any())

    def overlap(early):
        batch.materialize()
        got = early() if overlap_on and no_legacy else None
        if got is not None:
            prepared.append(chain.prepare_batch(batch, adjusted_time, got[0], got[1]))

    r = v.run(params, batch, series, plan, world, overlap=overlap)
    t1 = time.perf_counter()
    codes = r["codes"]
    n = len(batch)
    legacy = np.flatnonzero(codes == 255)
    hashes = r["hashes"]
    if len(legacy):  # X16R / X16RV2 headers (x16r_hashes: this device or the host cores), joined in
        hs = [batch.header(int(i)) for i in legacy]
        hashes = np.array(hashes)
        codes = np.array(codes)
        xs = x16r_hashes(params, [hdr.legacy80() for hdr in hs], [hdr.time for hdr in hs], device)
        for i, hdr, hsh in zip(legacy.tolist(), hs, xs):
            hashes[i] = np.frombuffer(hsh, np.uint8)
            ok = _core.check_proof_of_work(hsh, hdr.bits, params)
            codes[i] = 0 if ok else 2
    bad = np.flatnonzero(codes != 0)
    first_bad = int(bad[0]) if len(bad) else n
    t2 = time.perf_counter()
    if prepared:
        accepted, why, _dos = chain.commit_batch(prepared[0], first_bad)
    else:
        accepted, why, _dos = chain.accept_batch(batch, adjusted_time, hashes, r["bits"], 0, first_bad)
    t3 = time.perf_counter()
    reject = {"index": accepted, "reason": why} if why is not None else None
    if reject is None and first_bad < n:
        reject = {"index": first_bad, "reason": CODES.get(int(codes[first_bad]), "high-hash")}
    return {"accepted": accepted, "reject": reject, "dos": _dos, "pow_s": t1 - t0 + (t2 - t1), "context_s": t3 - t2,
            "dgw_gpu": series is not None, "resident": True,
            "sharded": world is not None and world.collective and world.world_size > 1,
            # host_ms: all host work (the wait for the device excluded); host_exposed_ms: the part
            # the device does not cover (the decode beside it counts only as far as the device ran
            # after the issue)
            "host_ms": round((t1 - t0) * 1e3 - r["wait_ms"] + (t3 - t1) * 1e3, 3),
            "host_exposed_ms": round((t1 - t0) * 1e3 - r["wait_ms"] + (t3 - t1) * 1e3
                                     - min(r["overlap_ms"], max(0.0, r["device_ms"] - r["issue_ms"])), 3),
            "overlap_ms": round(r["overlap_ms"], 3),
            "device_ms": round(r["device_ms"], 3), "pack_ms": round(r["pack_ms"], 3),
            "issue_ms": round(r["issue_ms"], 3), "wait_ms": round(r["wait_ms"], 3),
            "accept_ms": round((t3 - t2) * 1e3, 3)}
