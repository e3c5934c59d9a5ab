"""Batch X16R / X16RV2 hashing of legacy (80-byte) headers on the GPU.

Reference: HashX16R / HashX16RV2 (src/hash.h:335-605) hash one header at a time on the CPU, the
16-step algorithm order taken from hashPrevBlock (GetHashSelection, src/hash.h:320-327). Here a
whole batch advances one step per launch (hip/kernels/x16r.hip): the host groups the headers of
each step by the slot they run, once for the batch (`_core.x16r_groups`: a counting sort on each
step's selection nibble), and each step is one launch whose workgroup (x, slot) runs that slot over its group --
every wave executes one primitive. (One kernel per slot, a step's 16 groups on 4 fan-out streams,
measured 1.91 M against 2.27 M hashes/s: the groups are small and latency-bound, and 4 hardware
queues ran them at most 4 at a time; profiles/README r5k.) The 16 launches are queued by one
native call with the chain values resident on the device; one copy brings the 32-byte hashes back.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _core
from . import runtime


def selections(headers: np.ndarray) -> np.ndarray:
    """(n, 16) slot of each header at each step: nibble 48 + i of hashPrevBlock (header bytes
    4..35, storage order), as x16r_selection on the host."""
    prev = headers[:, 4:36]
    out = np.empty((len(headers), 16), dtype=np.int32)
    for i in range(16):
        j = 63 - (48 + i)
        byte = prev[:, j // 2]
        out[:, i] = (byte >> 4) if j % 2 == 1 else (byte & 0x0F)
    return out


def x16r_hash_batch(headers: bytes | np.ndarray, v2: bool | np.ndarray = False, device: int = 0) -> np.ndarray:
    """(n, 32) uint8 X16R (or, per header where `v2`, X16RV2) hashes of n 80-byte headers, in
    uint256 storage order (as `_core.x16r` / `_core.x16rv2` return them)."""
    runtime.require_gpu()
    hdr = np.frombuffer(headers, dtype=np.uint8) if isinstance(headers, (bytes, bytearray)) else np.asarray(headers, np.uint8)
    hdr = np.array(hdr.reshape(-1, 80), dtype=np.uint8, copy=True)  # writable, contiguous (torch.from_numpy)
    n = len(hdr)
    if n == 0:
        return np.zeros((0, 32), dtype=np.uint8)
    flags = np.broadcast_to(np.asarray(v2, dtype=np.uint8), (n,)).copy()
    # each step's slot groups: one native counting-sort pass per step (numpy's 16 argsorts took
    # several ms of host time per batch, as long as the kernels of a 16k batch)
    order_b, offsets = _core.x16r_groups(hdr)
    order = np.frombuffer(order_b, dtype=np.int32).reshape(16, n).copy()
    offsets = np.asarray(offsets, dtype=np.int32).reshape(16, 17)
    h = runtime.hip()
    dev = torch.device("cuda", device)
    with torch.cuda.device(dev):
        d_hdr = torch.from_numpy(hdr).to(dev)
        d_flags = torch.from_numpy(flags).to(dev)
        d_order = torch.from_numpy(order).to(dev)
        d_off = torch.from_numpy(offsets).to(dev)
        state = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        args = (d_hdr.data_ptr(), state.data_ptr(), d_flags.data_ptr(), d_order.data_ptr(), d_off.data_ptr(),
                offsets.reshape(-1).tolist(), n, runtime.current_stream_handle())
        h.launch_x16r_chain_all(runtime.static_kernel("x16r", "x16r_step_all"), *args)
        return state[:, :32].cpu().numpy()


class X16rSearcher:
    """GPU nonce search of a legacy header (generateBlocks' loop, src/rpc/mining.cpp:141-149, as
    `_core.x16r_search` does it on the host): every nonce of a window shares hashPrevBlock, so all
    of them run the same slot at each of the 16 steps -- one launch per step over the whole window
    -- and x16r_hits keeps the lowest nonce whose hash is <= the target."""

    def __init__(self, device: int = 0, window: int = 1 << 20):
        runtime.require_gpu()
        self.device = int(device)
        self.window = int(window)
        self.h = runtime.hip()
        self.slots = [runtime.static_kernel("x16r", f"x16r_step_{a}") for a in range(16)]
        self.hits = runtime.static_kernel("x16r", "x16r_hits")
        dev = torch.device("cuda", self.device)
        with torch.cuda.device(dev):
            self.state = torch.empty((self.window, 64), dtype=torch.uint8, device=dev)
            self.order = torch.arange(self.window, dtype=torch.int32, device=dev)
            self.offsets = torch.zeros((16, 17), dtype=torch.int32, device=dev)
            self.tmpl = torch.empty(80, dtype=torch.uint8, device=dev)
            self.best = torch.empty(1, dtype=torch.int32, device=dev)
        self.dev = dev

    def search(self, header80: bytes, v2: bool, target_le: bytes, start: int, count: int):
        """((nonce, hash) or None, hashes done): the lowest nonce in [start, start + count) whose
        X16R / X16RV2 hash (storage order) is <= target_le (little-endian uint256)."""
        if len(header80) != 80 or len(target_le) != 32:
            raise ValueError("80-byte header, 32-byte target")
        start &= 0xFFFFFFFF
        count = min(int(count), (1 << 32) - start)
        sel = selections(np.frombuffer(header80, dtype=np.uint8).reshape(1, 80))[0].tolist()
        offsets = np.zeros((16, 17), dtype=np.int32)
        done = 0
        with torch.cuda.device(self.dev):
            s = runtime.current_stream_handle()
            self.tmpl.copy_(torch.frombuffer(bytearray(header80), dtype=torch.uint8))
            while done < count:
                n = min(self.window, count - done)
                for k in range(16):
                    offsets[k, sel[k] + 1:] = n
                    offsets[k, :sel[k] + 1] = 0
                self.offsets.copy_(torch.from_numpy(offsets))
                self.best.fill_(-1)
                self.h.launch_x16r_search(self.slots, self.hits, self.tmpl.data_ptr(), self.state.data_ptr(),
                                          self.order.data_ptr(), self.offsets.data_ptr(), sel, start + done, n,
                                          bool(v2), bytes(target_le), self.best.data_ptr(), s)
                best = int(self.best.cpu().numpy().view(np.uint32)[0])
                if best != 0xFFFFFFFF:
                    return (start + done + best, bytes(self.state[best, :32].cpu().numpy().tobytes())), done + best + 1
                done += n
        return None, done
