"""GPU batch KawPow hashing for header verification (hip/kernels/kawpow_verify.hip).

Jobs are grouped by epoch (one resident DAG per epoch on the device) and,
inside an epoch, sorted by period and padded into 64-job slabs so that every
wave64 runs a single period's program (the kernel reads the op list as
wave-uniform data). One launch per epoch covers all periods of the batch.
"""
from __future__ import annotations

import struct
from collections import defaultdict

import torch

from .. import _core
from . import runtime
from .ethash import DeviceEpoch

_epochs: dict[tuple[int, int], DeviceEpoch] = {}
JOB = struct.Struct("<8IQII")


def _device_epoch(epoch: int, device: int) -> DeviceEpoch:
    key = (device, epoch)
    e = _epochs.get(key)
    if e is None:
        for k in [k for k in _epochs if k[0] == device]:  # keep one resident epoch per device here
            _epochs.pop(k)
        with torch.cuda.device(device):
            e = DeviceEpoch(epoch, device=device)
            e.build()
            torch.cuda.synchronize()
        _epochs[key] = e
    return e


def gpu_full_hash(block_numbers: list[int], header_hashes: list[bytes], nonces: list[int],
                  device: int = 0) -> list[tuple[bytes, bytes]]:
    """(final, mix) in ethash storage order for every job (full ProgPoW, DAG on the GPU)."""
    h = runtime.hip()
    out: list[tuple[bytes, bytes] | None] = [None] * len(nonces)
    by_epoch: dict[int, list[int]] = defaultdict(list)
    for i, bn in enumerate(block_numbers):
        by_epoch[bn // _core.EPOCH_LENGTH].append(i)
    kern = None
    for epoch, idxs in sorted(by_epoch.items()):
        ep = _device_epoch(epoch, device)
        with torch.cuda.device(device):
            if kern is None:
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
            buf = bytearray(JOB.size * len(order))
            for slot, i in enumerate(order):
                if i >= 0:
                    JOB.pack_into(buf, slot * JOB.size, *struct.unpack("<8I", header_hashes[i]), nonces[i],
                                  block_numbers[i], 0)
            jobs = torch.frombuffer(buf, dtype=torch.uint8).to(ep.device)
            progs = torch.tensor(programs, dtype=torch.int64).to(torch.int32).to(ep.device)
            slabs = torch.tensor(slab_prog, dtype=torch.int32, device=ep.device)
            res = torch.empty(len(order) * 16, dtype=torch.int32, device=ep.device)
            h.launch_kawpow_verify_batch(kern, ep.dag.data_ptr(), ep.items2048, jobs.data_ptr(), progs.data_ptr(),
                                         slabs.data_ptr(), len(order), res.data_ptr(), runtime.current_stream_handle())
            raw = res.cpu().numpy().tobytes()
        for slot, i in enumerate(order):
            if i >= 0:
                out[i] = (raw[slot * 64 + 32: slot * 64 + 64], raw[slot * 64: slot * 64 + 32])
    return out  # type: ignore[return-value]
