"""GPU batch KawPow hashing for header verification (BASELINE config 5).

Two kernels, chosen per epoch group of the batch:
  * "dag"   (hip/kernels/kawpow_verify.hip): the epoch DAG is resident in HBM
    (generated on the GPU, 0.15-0.6 s per epoch); jobs are sorted by period and
    padded into 64-job slabs so each wave64 runs one period's program with
    wave-uniform op fields. Best when the DAG is already resident (a mining
    node's current epoch) or for very large batches.
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
from collections import defaultdict

import torch

from .. import _core
from . import runtime
from .ethash import DeviceEpoch

_epochs: dict[tuple[int, int], DeviceEpoch] = {}        # (device, epoch) -> DAG-resident epochs
_light: dict[tuple[int, int], DeviceEpoch] = {}         # (device, epoch) -> light-only epochs
JOB = struct.Struct("<8IQII")
LIGHT_MAX_JOBS = 50_000


def _device_epoch(epoch: int, device: int) -> DeviceEpoch:
    key = (device, epoch)
    e = _epochs.get(key)
    if e is None:
        for k in [k for k in _epochs if k[0] == device]:  # keep one resident verify DAG per device
            _epochs.pop(k)
        with torch.cuda.device(device):
            e = DeviceEpoch(epoch, device=device)
            e.build()
            torch.cuda.synchronize()
        _epochs[key] = e
    return e


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
        _epochs[(epoch_dev.device.index, epoch_dev.epoch)] = epoch_dev


def _pack_jobs(order: list[int], header_hashes, nonces, block_numbers) -> bytearray:
    buf = bytearray(JOB.size * len(order))
    for slot, i in enumerate(order):
        if i >= 0:
            JOB.pack_into(buf, slot * JOB.size, *struct.unpack("<8I", header_hashes[i]), nonces[i], block_numbers[i], 0)
    return buf


def _run_dag(ep: DeviceEpoch, idxs, block_numbers, header_hashes, nonces, out) -> None:
    """Resident-DAG batch: one job per 16-lane group with its period's program staged in LDS
    (kawpow_verify_dag), so headers of thousands of different periods share one dense launch."""
    h = runtime.hip()
    kern = runtime.static_kernel("kawpow_verify_light", "kawpow_verify_dag")
    periods = sorted({block_numbers[i] // 3 for i in idxs})
    pidx = {p: k for k, p in enumerate(periods)}
    programs = [w for p in periods for w in _core.kawpow_program_words(p)]
    job_prog = [pidx[block_numbers[i] // 3] for i in idxs]
    assert max(job_prog) < len(periods) and len(programs) == 64 * len(periods)
    jobs = torch.frombuffer(_pack_jobs(list(idxs), header_hashes, nonces, block_numbers),
                            dtype=torch.uint8).to(ep.device)
    progs = torch.tensor(programs, dtype=torch.int64).to(torch.int32).to(ep.device)
    jp = torch.tensor(job_prog, dtype=torch.int32, device=ep.device)
    res = torch.empty(len(idxs) * 16, dtype=torch.int32, device=ep.device)
    h.launch_kawpow_verify_dag(kern, ep.dag.data_ptr(), ep.items2048, ep.l1.data_ptr(), jobs.data_ptr(),
                               progs.data_ptr(), len(periods), jp.data_ptr(), len(idxs), res.data_ptr(),
                               runtime.current_stream_handle())
    raw = res.cpu().numpy().tobytes()
    for slot, i in enumerate(idxs):
        out[i] = (raw[slot * 64 + 32: slot * 64 + 64], raw[slot * 64: slot * 64 + 32])


def _run_dag_slabs(ep: DeviceEpoch, idxs, block_numbers, header_hashes, nonces, out) -> None:
    """Wave-uniform variant (kawpow_verify_batch): jobs padded into 64-job single-period
    slabs. Efficient when each period has many jobs (nonce scans); kept as mode "dag-slab"."""
    h = runtime.hip()
    kern = runtime.static_kernel("kawpow_verify", "kawpow_verify_batch")
    by_period: dict[int, list[int]] = defaultdict(list)
    for i in idxs:
        by_period[block_numbers[i] // 3].append(i)
    programs, slab_prog, order = [], [], []
    for pi, (period, members) in enumerate(sorted(by_period.items())):
        programs.extend(_core.kawpow_program_words(period))
        padded = members + [-1] * ((-len(members)) % 64)
        order.extend(padded)
        slab_prog.extend([pi] * (len(padded) // 64))
    # the kernel indexes job_program[slot // 64] and programs[job_program * 64]
    assert len(slab_prog) * 64 == len(order) and max(slab_prog) < len(programs) // 64
    jobs = torch.frombuffer(_pack_jobs(order, header_hashes, nonces, block_numbers), dtype=torch.uint8).to(ep.device)
    progs = torch.tensor(programs, dtype=torch.int64).to(torch.int32).to(ep.device)
    slabs = torch.tensor(slab_prog, dtype=torch.int32, device=ep.device)
    res = torch.empty(len(order) * 16, dtype=torch.int32, device=ep.device)
    h.launch_kawpow_verify_batch(kern, ep.dag.data_ptr(), ep.items2048, jobs.data_ptr(), progs.data_ptr(),
                                 slabs.data_ptr(), len(order), res.data_ptr(), runtime.current_stream_handle())
    raw = res.cpu().numpy().tobytes()
    for slot, i in enumerate(order):
        if i >= 0:
            out[i] = (raw[slot * 64 + 32: slot * 64 + 64], raw[slot * 64: slot * 64 + 32])


def _run_light(ep: DeviceEpoch, idxs, block_numbers, header_hashes, nonces, out) -> None:
    h = runtime.hip()
    kern = runtime.static_kernel("kawpow_verify_light", "kawpow_verify_light")
    periods = sorted({block_numbers[i] // 3 for i in idxs})
    pidx = {p: k for k, p in enumerate(periods)}
    programs = [w for p in periods for w in _core.kawpow_program_words(p)]
    job_prog = [pidx[block_numbers[i] // 3] for i in idxs]
    assert max(job_prog) < len(periods) and len(programs) == 64 * len(periods)
    jobs = torch.frombuffer(_pack_jobs(list(idxs), header_hashes, nonces, block_numbers),
                            dtype=torch.uint8).to(ep.device)
    progs = torch.tensor(programs, dtype=torch.int64).to(torch.int32).to(ep.device)
    jp = torch.tensor(job_prog, dtype=torch.int32, device=ep.device)
    res = torch.empty(len(idxs) * 16, dtype=torch.int32, device=ep.device)
    h.launch_kawpow_verify_light(kern, ep.light.data_ptr(), int(ep.ctx.light_items), ep.l1.data_ptr(), ep.items2048,
                                 jobs.data_ptr(), progs.data_ptr(), len(periods), jp.data_ptr(), len(idxs),
                                 res.data_ptr(), runtime.current_stream_handle())
    raw = res.cpu().numpy().tobytes()
    for slot, i in enumerate(idxs):
        out[i] = (raw[slot * 64 + 32: slot * 64 + 64], raw[slot * 64: slot * 64 + 32])


def gpu_full_hash(block_numbers: list[int], header_hashes: list[bytes], nonces: list[int],
                  device: int = 0, mode: str = "auto") -> list[tuple[bytes, bytes]]:
    """(final, mix) in ethash storage order for every job (full ProgPoW on the GPU).

    mode: "dag" (build/reuse the epoch DAG), "light" (recompute items from the light
    cache) or "auto"."""
    if mode not in ("auto", "dag", "dag-slab", "light"):
        raise ValueError(f"unknown verify mode {mode}")
    out: list[tuple[bytes, bytes] | None] = [None] * len(nonces)
    by_epoch: dict[int, list[int]] = defaultdict(list)
    for i, bn in enumerate(block_numbers):
        by_epoch[bn // _core.EPOCH_LENGTH].append(i)
    for epoch, idxs in sorted(by_epoch.items()):
        m = mode
        if m == "auto":
            m = "dag" if (device, epoch) in _epochs or len(idxs) > LIGHT_MAX_JOBS else "light"
        with torch.cuda.device(device):
            if m == "dag":
                _run_dag(_device_epoch(epoch, device), idxs, block_numbers, header_hashes, nonces, out)
            elif m == "dag-slab":
                _run_dag_slabs(_device_epoch(epoch, device), idxs, block_numbers, header_hashes, nonces, out)
            else:
                _run_light(_light_epoch(epoch, device), idxs, block_numbers, header_hashes, nonces, out)
    return out  # type: ignore[return-value]


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
