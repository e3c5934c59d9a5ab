"""Batch SHA-256d on the GPU (hip/kernels/sha256d.hip).

`sha256d_batch` hashes many equal-length messages (block headers) one lane each;
`merkle_root` runs ComputeMerkleRoot (src/consensus/merkle.cpp) level by level on the
device, the nodes staying resident in HBM between levels. Digests are in the byte order
of the reference's CHash256 / uint256 storage (`_core.sha256d`)."""
from __future__ import annotations

import numpy as np
import torch

from . import runtime


def sha256d_batch(msgs, device: int = 0) -> np.ndarray:
    """(n, 32) uint8 digests of an (n, L) uint8 array (or a list of equal-length bytes)."""
    if not isinstance(msgs, np.ndarray):
        lens = {len(m) for m in msgs}
        if len(lens) > 1:
            raise ValueError("sha256d_batch needs equal-length messages")
        msgs = np.frombuffer(bytearray(b"".join(msgs)), dtype=np.uint8).reshape(len(msgs), -1) if msgs else \
            np.zeros((0, 0), np.uint8)
    n, length = msgs.shape
    if n == 0:
        return np.zeros((0, 32), np.uint8)
    dev = torch.device("cuda", device)
    with torch.cuda.device(device):
        d_in = torch.from_numpy(np.ascontiguousarray(msgs)).to(dev)
        d_out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        runtime.hip().launch_sha256d(runtime.static_kernel("sha256d", "sha256d_batch"), d_in.data_ptr(), length,
                                     length, n, d_out.data_ptr(), False, runtime.current_stream_handle())
        return d_out.cpu().numpy()


def merkle_root(txids: list[bytes], device: int = 0) -> bytes:
    """Merkle root of txids (uint256 storage order), last node duplicated on odd levels."""
    if not txids:
        return bytes(32)
    dev = torch.device("cuda", device)
    k = runtime.static_kernel("sha256d", "sha256d_merkle_level")
    with torch.cuda.device(device):
        cur = torch.from_numpy(np.frombuffer(b"".join(txids), dtype=np.uint8).copy()).to(dev)
        n = len(txids)
        while n > 1:
            m = (n + 1) // 2
            nxt = torch.empty(m * 32, dtype=torch.uint8, device=dev)
            runtime.hip().launch_sha256d(k, cur.data_ptr(), n, 32, m, nxt.data_ptr(), True,
                                         runtime.current_stream_handle())
            cur, n = nxt, m
        return cur.cpu().numpy().tobytes()


def kawpow_mixonly_batch(raw: np.ndarray, device: int = 0) -> np.ndarray:
    """(n, 128) rows for an (n, 120) uint8 array of KawPow headers: header hash | mix-only final |
    nBits boundary | claimed mix, ProgPoW byte order (hash_no_verify fused with the SHA256d header
    hash, hip/kernels/sha256d.hip: kawpow_mixonly_batch)."""
    n = len(raw)
    if n == 0:
        return np.zeros((0, 128), np.uint8)
    if raw.shape[1] != 120:
        raise ValueError("KawPow headers are 120 bytes")
    dev = torch.device("cuda", device)
    with torch.cuda.device(device):
        d_in = torch.from_numpy(np.ascontiguousarray(raw)).to(dev)
        d_out = torch.empty((n, 128), dtype=torch.uint8, device=dev)
        runtime.hip().launch_kawpow_mixonly(runtime.static_kernel("sha256d", "kawpow_mixonly_batch"), d_in.data_ptr(),
                                            n, 120, d_out.data_ptr(), runtime.current_stream_handle())
        return d_out.cpu().numpy()
