"""Pipelined KawPow nonce search on one device — the loop the node mines with and bench.py times.

Reference behaviour: the miner's inner loop (CloreMiner, src/miner.cpp:566-726: search, check
for a stale tip, count hashes) and progpow::search (src/crypto/ethash/lib/ethash/progpow.cpp:
553-579). The MI355X form differs in three ways that matter for throughput:

* **Big windows, two result slots.** Each launch searches 2^25 nonces (about 120 ms at epoch
  384: ~43k workgroups, far past the 512 that fill the chip). The device owns two share rings;
  the host queues window k+1 before it reads window k, and each ring is copied to pinned host
  memory on the search stream right behind its kernel, so the GPU is never idle waiting for the
  host and the host never blocks on the kernel it just queued.
* **Stale-work abort on the device.** Every launch carries a generation number; the device
  reads a host-mapped generation word once per workgroup (kawpow_search.hip). `abort()` bumps
  the word when the template changes, so queued work of the old template stops within one
  workgroup's lifetime (~1.4 ms) instead of finishing a 120 ms window. Workgroups that exit this
  way are counted in the ring (`skipped`), so the hash counter stays exact.
* **Shares are only candidates.** The kernel tests the top 64 bits of the final hash; the
  host applies the full 256-bit boundary and the miner fully re-hashes a share (light mode)
  before it builds a block from it (service.ChainLeader).

`CpuSearchDevice` runs the same protocol on the host (light-mode search, the reference's
search_light) so the multi-rank loop can be tested with the gloo backend on CPU-only machines.
"""
from __future__ import annotations

import struct
import threading
import time
from dataclasses import dataclass, field

from .. import core

_core = core()

# Work packet (collective #1): broadcast from rank 0 on every step of the mining loop.
#   header_hash 32 | boundary 32 (big-endian 256-bit target) | height u32 | epoch u32 |
#   job_id u64 | nonce_base u64 | flags u64  = 96 bytes
WORK_FMT = "<32s32sIIQQQ"
WORK_SIZE = struct.calcsize(WORK_FMT)
assert WORK_SIZE == 96

FLAG_IDLE = 1    # nothing to mine: drain and wait for the next packet
FLAG_STOP = 2    # leave the mining loop
FLAG_CLEAN = 4   # the previous job is stale: abort its queued work

EPOCH_PREBUILD_WINDOW = 120  # blocks before an epoch boundary at which the next DAG is prebuilt


@dataclass(frozen=True)
class Work:
    header_hash: bytes = bytes(32)   # KawPow header hash, progpow storage order
    boundary: bytes = bytes(32)      # share/block target, big-endian
    height: int = 0
    job_id: int = 0
    nonce_base: int = 0
    flags: int = FLAG_IDLE

    @property
    def epoch(self) -> int:
        return self.height // _core.EPOCH_LENGTH

    @property
    def idle(self) -> bool:
        return bool(self.flags & (FLAG_IDLE | FLAG_STOP))

    @property
    def stop(self) -> bool:
        return bool(self.flags & FLAG_STOP)

    def pack(self) -> bytes:
        return struct.pack(WORK_FMT, self.header_hash, self.boundary, self.height, self.epoch, self.job_id,
                           self.nonce_base, self.flags)

    @classmethod
    def unpack(cls, raw: bytes) -> "Work":
        hh, b, height, _epoch, job, base, flags = struct.unpack(WORK_FMT, raw)
        return cls(hh, b, height, job, base, flags)

    def target64(self) -> int:
        """Upper 64 bits of the boundary: the kernel's prefix test never rejects a hash the full
        256-bit compare would accept."""
        return int.from_bytes(self.boundary[:8], "big")


@dataclass
class SlotResult:
    """One finished window: the shares that pass the full 256-bit boundary and the nonces that
    were actually evaluated (an aborted window counts only the workgroups that ran)."""
    job_id: int
    start: int
    count: int
    hashes: int
    shares: list = field(default_factory=list)
    device_ms: float = 0.0


class DeviceHung(RuntimeError):
    """A window did not finish within the watchdog limit."""


class GpuSearchDevice:
    """One MI355X: resident epoch DAGs, per-period kernels, two share rings, the generation word.

    `collective_dag`: build DAGs sharded over the current process group and all-gather them
    (parallel/dag.py); every rank must then prepare the same epoch at the same step, which the
    mining service guarantees (all ranks act on the same broadcast work packet)."""

    name = "gpu"
    MAX_EPOCHS = 2  # current + next (two 4 GiB DAGs are ~3 % of 288 GB)

    def __init__(self, device: int = 0, collective_dag: bool = False):
        import torch

        from ..ops import runtime

        runtime.require_gpu()
        self.device = int(device)
        self.collective_dag = collective_dag
        self.h = runtime.hip()
        self.torch = torch
        self.epochs: dict[int, object] = {}
        self.searchers: dict[int, object] = {}
        self.lock = threading.Lock()
        nbytes = self.h.sizeof_results()
        with torch.cuda.device(self.device):
            self.stream = torch.cuda.Stream(device=self.device)
            self.side = torch.cuda.Stream(device=self.device)  # next-epoch DAG builds
            self.rings = [torch.zeros(nbytes // 4, dtype=torch.int32, device=self.device) for _ in range(2)]
            self.host = [torch.zeros(nbytes // 4, dtype=torch.int32).pin_memory() for _ in range(2)]
            self.events = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            self.starts = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        self.meta: list[tuple | None] = [None, None]
        self.gen_ptr = self.h.host_words_alloc(1)
        self.generation = 0
        self.pending_build: dict[int, object] = {}

    def close(self) -> None:
        if self.gen_ptr:
            self.torch.cuda.synchronize(self.device)
            self.h.host_words_free(self.gen_ptr)
            self.gen_ptr = 0

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ epochs / kernels
    def _build_epoch(self, epoch: int, stream=None):
        from ..ops.ethash import DeviceEpoch
        from ..parallel import dag as pdag
        from ..parallel import world as W

        torch = self.torch
        ws = W.get().world_size if self.collective_dag else 1
        with torch.cuda.device(self.device):
            e = DeviceEpoch(epoch, device=self.device, world_size=ws)
            with torch.cuda.stream(stream or self.stream):
                if self.collective_dag:
                    pdag.build_dag(e)
                else:
                    e.build()
        return e

    def epoch_ready(self, epoch: int) -> bool:
        return epoch in self.epochs

    def prebuild(self, epoch: int) -> None:
        """Queue epoch's DAG build on the side stream (collective when sharded; every rank calls this
        at the same step). The search stream keeps running; the epoch becomes usable once its build
        event has completed."""
        if epoch in self.epochs or epoch in self.pending_build:
            return
        torch = self.torch
        e = self._build_epoch(epoch, stream=self.side)
        with torch.cuda.device(self.device):
            ev = torch.cuda.Event()
            ev.record(self.side)
        self.pending_build[epoch] = (e, ev)

    def _epoch(self, epoch: int):
        if epoch in self.epochs:
            return self.epochs[epoch]
        torch = self.torch
        if epoch in self.pending_build:
            e, ev = self.pending_build.pop(epoch)
            self.stream.wait_event(ev)  # search kernels after the build, without a host sync
        else:
            e = self._build_epoch(epoch)
        with torch.cuda.device(self.device):
            self.stream.synchronize()
            if not e.l1_matches():
                raise RuntimeError(f"gpu{self.device}: epoch {epoch} DAG failed its L1 self-check")
        for old in [k for k in self.epochs if k < epoch - 1]:
            self.epochs.pop(old)
            self.searchers.pop(old, None)
        self.epochs[epoch] = e
        return e

    def searcher(self, height: int):
        from ..ops.kawpow import KawpowSearcher

        epoch = height // _core.EPOCH_LENGTH
        with self.lock:
            ep = self._epoch(epoch)
            s = self.searchers.get(epoch)
            if s is None:
                with self.torch.cuda.device(self.device):
                    s = KawpowSearcher(ep, height, prefetch_next=True)
                self.searchers[epoch] = s
            else:
                s.set_block(height)
            return s

    def block_for(self, height: int) -> int:
        return self.searcher(height).block

    # ------------------------------------------------------------------ the two slots
    def submit(self, slot: int, work: Work, start: int, count: int) -> None:
        torch = self.torch
        s = self.searcher(work.height)
        b = s.block
        count = max(b, count // b * b)
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            ring = self.rings[slot]
            ring[:4].zero_()
            self.starts[slot].record(self.stream)
            s.launch(work.header_hash, start, count, work.target64(), stream=int(self.stream.cuda_stream),
                     results=ring, gen_word=self.gen_ptr, generation=self.generation)
            self.host[slot].copy_(ring, non_blocking=True)
            self.events[slot].record(self.stream)
        self.meta[slot] = (work, start, count, b)

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        from ..ops.kawpow import parse_results

        ev = self.events[slot]
        if timeout_s is not None:
            deadline = time.monotonic() + timeout_s
            while not ev.query():
                if time.monotonic() > deadline:
                    raise DeviceHung(f"gpu{self.device}: search window did not finish in {timeout_s:.0f}s")
                time.sleep(0.0005)
        ev.synchronize()
        work, start, count, block = self.meta[slot]
        self.meta[slot] = None
        shares, _n, skipped = parse_results(self.host[slot].numpy().tobytes(), self.h.KAWPOW_MAX_SHARES)
        shares = [x for x in shares if _core.hash_le(x.final_hash, work.boundary)]
        hashes = max(0, count - skipped * block)
        return SlotResult(work.job_id, start, count, hashes, shares, self.starts[slot].elapsed_time(ev))

    def abort(self) -> None:
        """Make every queued or running window stale (its remaining workgroups exit at start)."""
        self.generation = (self.generation + 1) & 0xFFFFFFFF
        self.h.host_word_store(self.gen_ptr, 0, self.generation)

    def synchronize(self) -> None:
        self.stream.synchronize()


class CpuSearchDevice:
    """The same two-slot protocol on the host: light-mode search (progpow::search_light,
    src/crypto/ethash/lib/ethash/progpow.cpp:553-565), first share of each window. For CPU-only
    nodes and for rehearsing the multi-rank loop over gloo."""

    name = "cpu"
    device = -1

    def __init__(self, max_window: int = 4096):
        self.max_window = int(max_window)
        self.meta: list[tuple | None] = [None, None]
        self.generation = 0
        self.collective_dag = False

    def block_for(self, height: int) -> int:
        return 1

    def epoch_ready(self, epoch: int) -> bool:
        return True

    def prebuild(self, epoch: int) -> None:
        _core.get_epoch_context(epoch)

    def submit(self, slot: int, work: Work, start: int, count: int) -> None:
        self.meta[slot] = (work, start, min(count, self.max_window), self.generation)

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        from ..ops.kawpow import Share

        work, start, count, gen = self.meta[slot]
        self.meta[slot] = None
        if gen != self.generation:  # aborted before it ran
            return SlotResult(work.job_id, start, count, 0, [])
        t0 = time.perf_counter()
        ctx = _core.get_epoch_context(work.epoch)
        ok, nonce, fin, mix = _core.kawpow_search_light(ctx, work.height, work.header_hash, work.boundary,
                                                         start, count)
        dt = (time.perf_counter() - t0) * 1e3
        if ok:
            return SlotResult(work.job_id, start, count, nonce - start + 1, [Share(nonce, mix, fin)], dt)
        return SlotResult(work.job_id, start, count, count, [], dt)

    def abort(self) -> None:
        self.generation += 1

    def synchronize(self) -> None:
        pass

    def close(self) -> None:
        pass


class SearchPipeline:
    """Two windows in flight: `step` queues the next window, then returns the previous one's result.
    The device never waits for the host between windows; the host's share handling, collectives
    and bookkeeping overlap the window that is running."""

    def __init__(self, dev, watchdog_s: float | None = None):
        self.dev = dev
        self.watchdog_s = watchdog_s
        self.inflight: int | None = None
        self.next_slot = 0

    def step(self, work: Work, start: int, count: int) -> SlotResult | None:
        slot = self.next_slot
        self.dev.submit(slot, work, start, count)
        prev, self.inflight = self.inflight, slot
        self.next_slot ^= 1
        return self.dev.wait(prev, self.watchdog_s) if prev is not None else None

    def drain(self) -> SlotResult | None:
        if self.inflight is None:
            return None
        prev, self.inflight = self.inflight, None
        return self.dev.wait(prev, self.watchdog_s)


class HangingDevice:
    """Fault injection (tests, `NODEXA_MINER_HANG_AFTER`): behaves like `inner` for `after` windows,
    then every window hangs — wait() blocks until the watchdog limit and raises DeviceHung, which is
    what a GPU whose kernel never returns looks like to the mining loop."""

    def __init__(self, inner, after: int):
        self.inner = inner
        self.after = int(after)
        self.waits = 0

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        self.waits += 1
        if self.waits <= self.after:
            return self.inner.wait(slot, timeout_s)
        time.sleep(timeout_s if timeout_s is not None else 1e9)
        raise DeviceHung(f"{getattr(self.inner, 'name', 'dev')}: injected hang")
