"""GPU batch KawPow hashing for header verification (BASELINE config 5).

Three kernels, chosen per epoch group of the batch:
  * "dag"   (kawpow_verify_dag in hip/kernels/kawpow_verify_light.hip): the epoch
    DAG is resident in HBM (generated on the GPU, 0.15-0.6 s per epoch); one job per
    16-lane group with its period's program staged in LDS, so a batch spanning
    thousands of periods is one dense launch. Best when the DAG is already resident
    (a mining node's current epoch) or for very large batches.
  * "dag-slab" (kawpow_verify_batch in hip/kernels/kawpow_verify.hip): DAG-resident,
    jobs sorted by period and padded into 64-job slabs so each wave64 runs one
    period's program with wave-uniform op fields (nonce scans of one header).
  * "light" (hip/kernels/kawpow_verify_light.hip): no DAG; every 2048-bit item a
    hash touches is recomputed from the light cache (4 x 512 parents), one job
    per 16-lane group, any mix of periods per launch. Work per header is
    ~1/262k of a DAG build at epoch 384, so for header-sync batches (2000 per
    P2P `headers` message, 10k in the BASELINE config) it avoids the build.
`mode="auto"` uses a resident DAG when there is one and otherwise picks light
below LIGHT_MAX_JOBS jobs per epoch.
"""
from __future__ import annotations

import struct
import threading

import numpy as np
import torch

from .. import _core
from . import runtime
from .ethash import DeviceEpoch

_epochs: dict[tuple[int, int], DeviceEpoch] = {}        # (device, epoch) -> DAG-resident epochs
_light: dict[tuple[int, int], DeviceEpoch] = {}         # (device, epoch) -> light-only epochs
JOB = struct.Struct("<8IQII")
JOB_DT = np.dtype([("hh", "<u4", 8), ("nonce", "<u8"), ("bn", "<u4"), ("pad", "<u4")])
LIGHT_MAX_JOBS = 50_000
MAX_RESIDENT_DAGS = 4  # per device: <= 4 x ~5 GiB of the 288 GiB HBM
# the miner thread offers its DAGs (share_epoch) while the P2P thread verifies (_device_epoch):
# every access to _epochs holds this lock
_epochs_lock = threading.RLock()


def _device_epoch(epoch: int, device: int) -> DeviceEpoch:
    key = (device, epoch)
    with _epochs_lock:
        e = _epochs.get(key)
        if e is None:
            mine = [k for k in list(_epochs) if k[0] == device]  # LRU: a header batch often spans 2 epochs
            for k in mine[:max(0, len(mine) - MAX_RESIDENT_DAGS + 1)]:
                _epochs.pop(k)
            with torch.cuda.device(device):
                e = DeviceEpoch(epoch, device=device)
                e.build()
                torch.cuda.synchronize()
            _epochs[key] = e
        else:
            _epochs[key] = _epochs.pop(key)  # most recently used last
        return e


def is_resident(device: int, epoch: int) -> bool:
    with _epochs_lock:
        return (device, epoch) in _epochs


def share_epoch(device: int, epoch: int, e: DeviceEpoch) -> None:
    """Offer a DAG built elsewhere on `device` (the miner's, miner/search.GpuSearchDevice) to batch
    verify: a mining node then verifies the current epoch's headers against the DAG it mines on
    instead of building a second 4 GiB copy (read-only on both sides)."""
    with _epochs_lock:
        _epochs.setdefault((device, epoch), e)


def prefetch_contexts(epochs, device: int) -> None:
    """Build the host epoch contexts (light caches: a serial keccak chain per epoch, ~0.5 s at
    epoch 0 and ~2 s at 384 on one core) of the batch's epochs that this device has neither as a
    resident DAG nor as a light epoch, in parallel threads (the native build releases the GIL), so
    a batch that crosses an epoch boundary pays for one build, not two in a row. The native LRU
    (csrc/pow/ethash.cpp get_epoch_context) then hands them to DeviceEpoch."""
    with _epochs_lock:
        need = [int(e) for e in epochs if (device, int(e)) not in _epochs and (device, int(e)) not in _light]
    if len(need) > 1:
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(min(len(need), 4)) as ex:
            list(ex.map(_core.get_epoch_context, need[:4]))


def _light_epoch(epoch: int, device: int) -> DeviceEpoch:
    key = (device, epoch)
    e = _light.get(key)
    if e is None:
        if len(_light) >= 8:
            _light.pop(next(iter(_light)))
        with torch.cuda.device(device):
            e = DeviceEpoch(epoch, device=device, light_only=True)
        _light[key] = e
    return e


def register_resident(epoch_dev: DeviceEpoch) -> None:
    """Let verification reuse a DAG some other component (the miner) keeps resident."""
    if epoch_dev.built and epoch_dev.dag is not None:
        with _epochs_lock:
            _epochs[(epoch_dev.device.index, epoch_dev.epoch)] = epoch_dev


def _pack_jobs(block_numbers, header_hashes, nonces) -> np.ndarray:
    """(m, 48) uint8 job records (JOB) from per-job lists."""
    jobs = np.zeros(len(nonces), dtype=JOB_DT)
    if len(nonces):
        jobs["hh"] = np.frombuffer(b"".join(header_hashes), dtype="<u4").reshape(-1, 8)
        jobs["nonce"] = np.asarray(nonces, dtype=np.uint64)
        jobs["bn"] = np.asarray(block_numbers, dtype=np.uint32)
    return jobs.view(np.uint8).reshape(-1, JOB.size)


def _block_numbers(jobs: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(jobs[:, 40:44]).view("<u4").ravel()


def _programs(periods, device) -> torch.Tensor:
    raw = _core.kawpow_programs_bytes([int(p) for p in periods])
    assert len(raw) == 256 * len(periods)
    return torch.frombuffer(bytearray(raw), dtype=torch.int32).to(device)


def _grouped(jobs: np.ndarray, device):
    """Device job records, the program of every distinct period in the batch and each
    job's index into that program table (the kernels' job_program operand)."""
    periods, job_prog = np.unique(_block_numbers(jobs) // 3, return_inverse=True)
    dj = torch.from_numpy(np.ascontiguousarray(jobs)).to(device)
    jp = torch.from_numpy(job_prog.astype(np.int32).ravel()).to(device)
    return dj, _programs(periods, device), len(periods), jp


def _run_dag(ep: DeviceEpoch, jobs: np.ndarray):
    """Resident-DAG batch: one job per 16-lane group, headers of thousands of different periods in
    one dense launch. kawpow_verify_waves (jobs grouped by period four to a wave64, the program
    wave-uniform, the mix in VGPRs) unless the test hook header_batch.WAVES selects kawpow_verify_dag (each
    group's program and mix in LDS). Like the other _run_*: issued on the current stream, returns
    the call that waits for it and yields the (m, 64) rows."""
    from . import header_batch as HB

    m = len(jobs)
    dj, progs, nprog, jp = _grouped(jobs, ep.device)
    res = torch.empty(m * 16, dtype=torch.int32, device=ep.device)
    h = runtime.hip()
    if HB.WAVES:
        heights = np.ascontiguousarray(_block_numbers(jobs), dtype="<u4")
        slots = np.frombuffer(_core.wave_slots(np.zeros(m, dtype=np.uint8), heights, 0, m), dtype=np.int32)
        ds = torch.from_numpy(slots.copy()).to(ep.device)
        h.launch_kawpow_verify_waves(runtime.static_kernel("kawpow_verify_light", "kawpow_verify_waves"),
                                     ep.dag.data_ptr(), ep.items2048, ep.l1.data_ptr(), dj.data_ptr(),
                                     progs.data_ptr(), nprog, jp.data_ptr(), m, ds.data_ptr(), len(slots),
                                     res.data_ptr(), runtime.current_stream_handle())
    else:
        h.launch_kawpow_verify_dag(
            runtime.static_kernel("kawpow_verify_light", "kawpow_verify_dag"), ep.dag.data_ptr(), ep.items2048,
            ep.l1.data_ptr(), dj.data_ptr(), progs.data_ptr(), nprog, jp.data_ptr(), m, res.data_ptr(),
            runtime.current_stream_handle())
    return lambda: res.cpu().numpy().view(np.uint8).reshape(m, 64)


def _run_dag_slabs(ep: DeviceEpoch, jobs: np.ndarray) -> np.ndarray:
    """Wave-uniform variant (kawpow_verify_batch): jobs padded into 64-job single-period
    slabs. Efficient when each period has many jobs (nonce scans); kept as mode "dag-slab"."""
    per = _block_numbers(jobs) // 3
    srt = np.argsort(per, kind="stable")
    _, first, counts = np.unique(per[srt], return_index=True, return_counts=True)
    parts, slab_prog = [], []
    for k, (f, c) in enumerate(zip(first.tolist(), counts.tolist())):
        pad = (-c) % 64
        parts += [srt[f:f + c], np.full(pad, -1, dtype=np.int64)]
        slab_prog += [k] * ((c + pad) // 64)
    order = np.concatenate(parts)
    valid = order >= 0
    padded = np.zeros((len(order), JOB.size), dtype=np.uint8)
    padded[valid] = jobs[order[valid]]
    # the kernel indexes job_program[slot // 64] and programs[job_program * 64]
    assert len(slab_prog) * 64 == len(order) and max(slab_prog) < len(first)
    dj = torch.from_numpy(padded).to(ep.device)
    progs = _programs(np.unique(per), ep.device)
    slabs = torch.tensor(slab_prog, dtype=torch.int32, device=ep.device)
    res = torch.empty(len(order) * 16, dtype=torch.int32, device=ep.device)
    runtime.hip().launch_kawpow_verify_batch(
        runtime.static_kernel("kawpow_verify", "kawpow_verify_batch"), ep.dag.data_ptr(), ep.items2048,
        dj.data_ptr(), progs.data_ptr(), slabs.data_ptr(), len(order), res.data_ptr(),
        runtime.current_stream_handle())

    def finish():
        raw = res.cpu().numpy().view(np.uint8).reshape(len(order), 64)
        out = np.empty((len(jobs), 64), dtype=np.uint8)
        out[order[valid]] = raw[valid]
        return out

    return finish


def _run_light(ep: DeviceEpoch, jobs: np.ndarray):
    m = len(jobs)
    dj, progs, nprog, jp = _grouped(jobs, ep.device)
    res = torch.empty(m * 16, dtype=torch.int32, device=ep.device)
    runtime.hip().launch_kawpow_verify_light(
        runtime.static_kernel("kawpow_verify_light", "kawpow_verify_light"), ep.light.data_ptr(),
        int(ep.ctx.light_items), ep.l1.data_ptr(), ep.items2048, dj.data_ptr(), progs.data_ptr(), nprog,
        jp.data_ptr(), m, res.data_ptr(), runtime.current_stream_handle())
    return lambda: res.cpu().numpy().view(np.uint8).reshape(m, 64)


def gpu_hash_jobs(jobs: np.ndarray, device: int = 0, mode: str = "auto") -> np.ndarray:
    """Full ProgPoW of (m, 48) uint8 job records on one GPU -> (m, 64) uint8 rows:
    mix (bytes 0..31) then final (32..63), ethash storage order.

    mode: "dag" (build/reuse the epoch DAG, dense kernel), "dag-slab" (DAG, per-period
    slabs), "light" (recompute items from the light cache) or "auto"."""
    if mode not in ("auto", "dag", "dag-slab", "light"):
        raise ValueError(f"unknown verify mode {mode}")
    jobs = np.asarray(jobs, dtype=np.uint8).reshape(-1, JOB.size)
    out = np.empty((len(jobs), 64), dtype=np.uint8)
    epochs = _block_numbers(jobs) // _core.EPOCH_LENGTH
    # every epoch group is issued before any is waited for, each on a stream of its own: a launch
    # is bound by its jobs' 64 dependent rounds (light: 64 x 512 dependent light-cache reads,
    # ~14 ms at any batch size the GPU holds), so the groups of a batch that spans an epoch
    # boundary run side by side instead of one after the other
    groups = np.unique(epochs).tolist()
    prefetch_contexts(groups, device)
    with torch.cuda.device(device):
        # at most MAX_RESIDENT_DAGS groups in flight: every epoch of a wave is resolved (DAG built
        # or light cache uploaded) before its first launch and held until its read-back, so the
        # LRUs can never evict, and the allocator never reuse, a DAG or light cache that a launch
        # still in flight reads
        for lo in range(0, len(groups), MAX_RESIDENT_DAGS):
            wave = []
            for epoch in groups[lo:lo + MAX_RESIDENT_DAGS]:
                idx = np.flatnonzero(epochs == epoch)
                m = mode
                if m == "auto":
                    m = "dag" if is_resident(device, epoch) or len(idx) > LIGHT_MAX_JOBS else "light"
                wave.append((idx, m, _light_epoch(epoch, device) if m == "light" else _device_epoch(epoch, device)))
            pending = []
            for k, (idx, m, ep) in enumerate(wave):
                s = _side_stream(device, k)
                s.wait_stream(torch.cuda.current_stream(device))  # the epoch's uploads / build
                with torch.cuda.stream(s):
                    run = _run_dag if m == "dag" else _run_dag_slabs if m == "dag-slab" else _run_light
                    pending.append((idx, s, run(ep, jobs[idx])))
            for idx, s, finish in pending:
                with torch.cuda.stream(s):  # the read-back queues behind its own launch
                    out[idx] = finish()
            del wave, pending
    return out


_streams: dict[tuple[int, int], torch.cuda.Stream] = {}


def _side_stream(device: int, k: int) -> torch.cuda.Stream:
    """The k-th (mod 4) verify stream of `device`, made once: epoch groups of one batch."""
    key = (device, k % 4)
    s = _streams.get(key)
    if s is None:
        s = _streams[key] = torch.cuda.Stream(device=device)
    return s


def gpu_full_hash(block_numbers: list[int], header_hashes: list[bytes], nonces: list[int],
                  device: int = 0, mode: str = "auto") -> list[tuple[bytes, bytes]]:
    """(final, mix) in ethash storage order for every job (list form of gpu_hash_jobs)."""
    raw = gpu_hash_jobs(_pack_jobs(block_numbers, header_hashes, nonces), device=device, mode=mode)
    return [(r[32:].tobytes(), r[:32].tobytes()) for r in raw]


class DagNonceScanner:
    """Period-agnostic nonce scan over one header on the DAG-resident verify kernel.

    Used where a header's period changes every few calls (synthetic chain mining:
    one new header per search), so per-period JIT kernels (ops/kawpow.py) would
    spend seconds compiling for a few thousand hashes. Job records are packed with
    numpy and the device buffers are reused, so one call costs one launch + one
    128 KiB read-back; the first final <= boundary in nonce order is returned."""

    def __init__(self, device: int = 0, width: int = 2048):
        import numpy as np

        assert width % 64 == 0
        self.np, self.device, self.width = np, device, width
        self.dt = np.dtype([("hh", "<u4", 8), ("nonce", "<u8"), ("bn", "<u4"), ("pad", "<u4")])
        assert self.dt.itemsize == JOB.size
        with torch.cuda.device(device):
            self.res = torch.empty(width * 16, dtype=torch.int32, device=f"cuda:{device}")
            self.slabs = torch.zeros(width // 64, dtype=torch.int32, device=f"cuda:{device}")
        self._prog_period = None
        self._progs = None

    def __call__(self, height: int, header_hash: bytes, boundary: bytes, start: int):
        np = self.np
        ep = _device_epoch(height // _core.EPOCH_LENGTH, self.device)
        period = height // 3
        with torch.cuda.device(self.device):
            if self._prog_period != period:
                self._progs = torch.tensor(_core.kawpow_program_words(period), dtype=torch.int64).to(
                    torch.int32).to(ep.device)
                self._prog_period = period
            jobs = np.zeros(self.width, dtype=self.dt)
            jobs["hh"] = np.frombuffer(header_hash, dtype="<u4")
            jobs["nonce"] = np.arange(start, start + self.width, dtype=np.uint64)
            jobs["bn"] = height
            dj = torch.from_numpy(jobs.view(np.uint8)).to(ep.device)
            runtime.hip().launch_kawpow_verify_batch(
                runtime.static_kernel("kawpow_verify", "kawpow_verify_batch"), ep.dag.data_ptr(), ep.items2048,
                dj.data_ptr(), self._progs.data_ptr(), self.slabs.data_ptr(), self.width, self.res.data_ptr(),
                runtime.current_stream_handle())
            raw = self.res.cpu().numpy().view(np.uint8).reshape(self.width, 64)
        # final = bytes 32..63 in storage (big-endian compare) order: test the top 8 bytes first
        top = raw[:, 32:40].copy().view(">u8").ravel()
        bound_top = int.from_bytes(boundary[:8], "big")
        for slot in np.nonzero(top <= bound_top)[0]:
            fin = raw[slot, 32:64].tobytes()
            if _core.hash_le(fin, boundary):
                return (start + int(slot), fin, raw[slot, 0:32].tobytes()), self.width
        return None, self.width
