"""Batch ECDSA (secp256k1) verification on the GPU (hip/kernels/secp256k1_verify.hip).

The reference checks every input signature serially on the CPU, spread over its script-check
thread pool (CCheckQueue, src/checkqueue.h:33-160; CPubKey::Verify, src/pubkey.cpp:169). Here a
block's (or a mempool batch's) signatures are collected as (pubkey, DER signature, message hash)
triples (chain/interpreter.hpp PendingSig), packed by the native core (`_core.secp_pack_jobs`),
and verified one per GPU thread. Verdicts 2 ("degenerate addition") are re-checked on the host
with the golden model, so the GPU result always equals CPubKey::Verify's.
"""
from __future__ import annotations

import threading

import torch

from .. import _core
from ..utils.trace import traced
from . import runtime

_tables: dict[int, torch.Tensor] = {}
_lock = threading.Lock()


def _gen_table(dev: torch.device) -> torch.Tensor:
    """The 64 KiB comb table of G, resident once per device."""
    with _lock:
        t = _tables.get(dev.index)
        if t is None:
            t = torch.frombuffer(bytearray(_core.secp_gen_table32()), dtype=torch.int32).to(dev)
            _tables[dev.index] = t
        return t


@traced("secp.verify_batch")
def verify_batch(items: list[tuple[bytes, bytes, bytes]], device: int | None = None) -> list[bool]:
    """items: (public key, DER signature without the hash-type byte, 32-byte message).
    Returns CPubKey::Verify's answer for each (lax DER, high S accepted)."""
    if not items:
        return []
    runtime.require_gpu()
    h = runtime.hip()
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else int(device))
    packed = _core.secp_pack_jobs(list(items))
    with torch.cuda.device(dev):
        kern = runtime.static_kernel("secp256k1_verify", "secp_verify_batch")
        jobs = torch.frombuffer(bytearray(packed), dtype=torch.int32).to(dev, non_blocking=False)
        out = torch.empty(len(items), dtype=torch.int32, device=dev)
        h.launch_secp_verify(kern, jobs.data_ptr(), len(items), _gen_table(dev).data_ptr(), out.data_ptr(),
                             runtime.current_stream_handle())
        verdicts = out.cpu().tolist()
    res = []
    for (pub, sig, msg), v in zip(items, verdicts):
        if v == 2:  # a doubling / inverse case inside an addition: the host decides
            res.append(bool(_core.secp_verify(pub, sig, msg)))
        else:
            res.append(v == 1)
    return res
