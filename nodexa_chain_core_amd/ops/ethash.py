"""Ethash epoch state resident on one MI355X: light cache + full DAG.

The light cache is built on the host (inherently serial keccak chain,
SURVEY K5) by `_core` and uploaded once; the DAG is generated on the GPU by
`ethash_dag_build` (hip/kernels/ethash_dag.hip) straight into a torch-owned
buffer. A 4 GiB DAG is 1.4 % of one GPU's 288 GB HBM3E, so several epochs can
stay resident (next-epoch prebuild, cross-epoch batch verification).

For multi-GPU nodes `build(shard=(rank, world))` computes only this rank's
contiguous slice in place; parallel/dag.py then all-gathers the slices over
RCCL ("DAG sharding").
"""
from __future__ import annotations

import torch

from .. import _core
from . import runtime
from ..utils.trace import traced

# 512-bit items per launch: keeps a single dispatch well under a second even
# at epoch 384 while still giving >> 256 CUs x 8 waves of work.
_DAG_CHUNK = 1 << 22
# hashes per 16-lane row of ethash_hash_batch (EH_HASHES in hip/kernels/ethash_hashimoto.hip)
EH_HASHES = 2


class DeviceEpoch:
    def __init__(self, epoch: int, device: int | torch.device | None = None, ctx=None, world_size: int = 1,
                 light_only: bool = False):
        """`light_only`: keep just the light cache and the 16 KiB L1 on the device (light-mode
        batch verification, ops/verify.py) — no DAG allocation."""
        runtime.require_gpu()
        self.epoch = int(epoch)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   (device.index if isinstance(device, torch.device) else int(device)))
        self.ctx = ctx if ctx is not None else _core.get_epoch_context(self.epoch)
        self.full_items = int(self.ctx.full_items)          # 1024-bit items
        self.items512 = 2 * self.full_items
        self.items2048 = self.full_items // 2
        self.dag_bytes = self.items512 * 64
        with torch.cuda.device(self.device):
            self.light = torch.empty(int(self.ctx.light_bytes), dtype=torch.uint8, device=self.device)
            runtime.hip().memcpy_htod(self.light.data_ptr(), self.ctx.light_cache_ptr(), int(self.ctx.light_bytes))
            self.l1 = torch.tensor(self.ctx.l1, dtype=torch.int64).to(torch.int32).to(self.device)
            if light_only:
                self._storage = None
                self.dag = None
            else:
                # padded to a whole number of equal shards so RCCL can all-gather in place
                self._storage = torch.empty(self.shard_bytes(world_size) * world_size, dtype=torch.uint8,
                                            device=self.device)
                self.dag = self._storage[:self.dag_bytes]
        self.built = False

    # ------------------------------------------------------------------
    def shard_items(self, world: int) -> int:
        return (self.items512 + world - 1) // world

    def shard_bytes(self, world: int) -> int:
        return self.shard_items(world) * 64

    def dag_padded(self, world: int) -> torch.Tensor:
        n = self.shard_bytes(world) * world
        if n > self._storage.numel():
            raise ValueError("DeviceEpoch was allocated for a smaller world size")
        return self._storage[:n]

    def shard_range(self, rank: int, world: int) -> tuple[int, int]:
        """[first, first+count) 512-bit items owned by `rank` (equal contiguous slices)."""
        per = self.shard_items(world)
        first = min(rank * per, self.items512)
        return first, min(per, self.items512 - first)

    @traced("ethash.dag_build")
    def build(self, shard: tuple[int, int] | None = None, stream: int | None = None) -> None:
        if self.dag is None:
            raise ValueError("light-only DeviceEpoch has no DAG to build")
        h = runtime.hip()
        with torch.cuda.device(self.device):
            k = runtime.static_kernel("ethash_dag", "ethash_dag_build")
            s = runtime.current_stream_handle() if stream is None else stream
            first, count = (0, self.items512) if shard is None else self.shard_range(*shard)
            end = first + count
            pos = first
            while pos < end:
                n = min(_DAG_CHUNK, end - pos)
                h.launch_ethash_dag_build(k, self.light.data_ptr(), int(self.ctx.light_items), self.dag.data_ptr(),
                                          pos, n, s)
                pos += n
        if shard is None:
            self.built = True

    def mark_built(self) -> None:
        self.built = True

    def l1_matches(self) -> bool:
        """The first 16 KiB of the device DAG equals the host-computed KawPow L1."""
        dev = self.dag[:16384].cpu().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        ref = torch.tensor(self.ctx.l1, dtype=torch.int64)
        return bool(torch.equal(dev, ref))

    def item512(self, index: int) -> bytes:
        return bytes(self.dag[index * 64:(index + 1) * 64].cpu().numpy().tobytes())

    def hashimoto_batch(self, header_hashes: list[bytes], nonces: list[int], stream: int | None = None
                        ) -> list[tuple[bytes, bytes]]:
        """Classic Ethash (final_hash, mix_hash) of each (header hash, nonce) over this resident
        DAG (hip/kernels/ethash_hashimoto.hip; ethash::hash, src/crypto/ethash/lib/ethash/
        ethash.cpp:416-440), as `_core.ethash_hash` computes them on the host."""
        import struct

        if not self.built or self.dag is None:
            raise RuntimeError("hashimoto_batch needs the built DAG")
        n = len(nonces)
        if n != len(header_hashes):
            raise ValueError("one nonce per header hash")
        if n == 0:
            return []
        job = struct.Struct("<8IQII")
        buf = bytearray(job.size * n)
        for i, (hh, nonce) in enumerate(zip(header_hashes, nonces)):
            if len(hh) != 32:
                raise ValueError("header hashes are 32 bytes")
            job.pack_into(buf, i * job.size, *struct.unpack("<8I", hh), int(nonce), 0, 0)
        h = runtime.hip()
        ks = [runtime.static_kernel("ethash_hashimoto", f"ethash_{x}_batch") for x in ("seed", "mix", "final")]
        with torch.cuda.device(self.device):
            jobs = torch.frombuffer(buf, dtype=torch.uint8).to(self.device)
            out = torch.empty(n * 16, dtype=torch.int32, device=self.device)
            seeds = torch.empty(n * 16, dtype=torch.int32, device=self.device)
            s = runtime.current_stream_handle() if stream is None else stream
            h.launch_ethash_hash_batch(*ks, self.dag.data_ptr(), self.full_items, jobs.data_ptr(), n, out.data_ptr(),
                                       seeds.data_ptr(), s, EH_HASHES)
            raw = out.cpu().numpy().tobytes()
        return [(raw[i * 64 + 32:i * 64 + 64], raw[i * 64:i * 64 + 32]) for i in range(n)]

    def ethash_search(self, header_hash: bytes, boundary: bytes, start_nonce: int, iterations: int,
                      window: int = 1 << 22) -> tuple[int, bytes, bytes] | None:
        """ethash::search (src/crypto/ethash/lib/ethash/ethash.cpp:326-350): the first nonce in
        [start_nonce, start_nonce + iterations) whose classic Ethash final hash is <= boundary, as
        (nonce, final_hash, mix_hash), or None. Nonces run on the device in windows of `window`
        (job i = start + i, no host-side job list); the final kernel appends each hit and the
        lowest one of the first window that has any is the answer."""
        if not self.built or self.dag is None:
            raise RuntimeError("ethash_search needs the built DAG")
        if len(header_hash) != 32 or len(boundary) != 32:
            raise ValueError("32-byte header hash and boundary")
        h = runtime.hip()
        ks = [runtime.static_kernel("ethash_hashimoto", f"ethash_{x}_batch") for x in ("seed", "mix", "final")]
        max_hits = 1024
        with torch.cuda.device(self.device):
            w = max(1, min(int(window), int(iterations)))
            out = torch.empty(w * 16, dtype=torch.int32, device=self.device)
            seeds = torch.empty(w * 16, dtype=torch.int32, device=self.device)
            hits = torch.zeros(1 + max_hits, dtype=torch.int32, device=self.device)
            s = runtime.current_stream_handle()
            done = 0
            while done < iterations:
                n = min(w, iterations - done)
                start = (int(start_nonce) + done) & 0xFFFFFFFFFFFFFFFF
                hits.zero_()
                h.launch_ethash_hash_batch(*ks, self.dag.data_ptr(), self.full_items, 0, n, out.data_ptr(),
                                           seeds.data_ptr(), s, EH_HASHES, bytes(header_hash), start, bytes(boundary),
                                           hits.data_ptr(), max_hits)
                got = hits.cpu().numpy().view("<u4")
                cnt = int(got[0])
                if cnt:
                    i = int(got[1:1 + min(cnt, max_hits)].min())
                    if cnt > max_hits:  # the ring overflowed: the lowest hit may be past it
                        raw = out[:n * 16].cpu().numpy().tobytes()
                        i = next(j for j in range(n) if raw[j * 64 + 32:j * 64 + 64] <= boundary)
                    row = out[i * 16:(i + 1) * 16].cpu().numpy().tobytes()
                    return (start + i) & 0xFFFFFFFFFFFFFFFF, row[32:], row[:32]
                done += n
        return None
