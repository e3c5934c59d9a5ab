"""Pipelined nonce search on one device — the loop the node mines with and bench.py times.

Reference behaviour: the miner's inner loop (CloreMiner, src/miner.cpp:566-726: search, check
for a stale tip, count hashes), progpow::search (src/crypto/ethash/lib/ethash/progpow.cpp:
553-579) and generateBlocks' legacy nNonce scan (src/rpc/mining.cpp:141-149). One work packet
format and one two-slot device protocol carry every proof of work the chain knows:

* **KawPow** (GpuSearchDevice / CpuSearchDevice). Each GPU launch searches 2^25 nonces (~120 ms at
  epoch 384: ~43k workgroups, far past the 512 that fill the chip). The device owns two share
  rings; the host queues window k+1 before it reads window k, and each ring is copied to pinned
  host memory on the search stream right behind its kernel, so the GPU is never idle waiting for
  the host. Every launch carries a generation number that the kernel reads once per workgroup from
  a host-mapped word: `abort()` bumps it when the template changes, so queued work of the old
  template stops within one workgroup's lifetime (~1.4 ms). The kernel tests the top 64 bits of the
  final hash; the host applies the full 256-bit boundary and the leader fully re-hashes a share
  (light mode) before it builds a block from it (service.ChainLeader).
* **Equihash(200,9)** (miner/equihash_search.py). A window is `count` nonce256 values
  (le64(nonce) || 24 zero bytes) appended to the 80-byte header prefix; the GPU solves them in one
  launch sequence, verifies every solution on the device and the host keeps the solutions whose
  SHA256d(header) meets the boundary.
* **X16R / X16RV2** (LegacyGpuDevice on a GPU rank, LegacyHostDevice otherwise): templates before
  the KawPow activation (the default on regtest) scan the 32-bit nNonce, 2^20 nonces per GPU
  window (hip/kernels/x16r.hip, search mode) or 2^16 on the host cores (csrc/pow/x16r.cpp).

`RankDevice` routes each slot to the device of its work packet's algorithm, so one loop, one set
of collectives and one failure path serve every era of the chain; `FaultInjectingDevice`
(-gpufailrate / -dropshare) and `HangingDevice` wrap any of them for the failure tests.
"""
from __future__ import annotations

import hashlib
import struct
import threading
import time
from dataclasses import dataclass, field

from .. import core

_core = core()

# Work packet (collective #1): broadcast from rank 0 on every step of the mining loop.
#   header 80 (KawPow: the header hash in bytes 0..31; Equihash: the 80-byte CKAWPOWInput-layout
#   prefix the nonce256 is appended to; X16R: the 80-byte legacy header with nNonce 0) |
#   boundary 32 (big-endian 256-bit target) | height u32 | algo u32 | job_id u64 |
#   nonce_base u64 | flags u64  = 144 bytes
WORK_FMT = "<80s32sIIQQQ"
WORK_SIZE = struct.calcsize(WORK_FMT)
assert WORK_SIZE == 144

FLAG_IDLE = 1    # nothing to mine: drain and wait for the next packet
FLAG_STOP = 2    # leave the mining loop
FLAG_CLEAN = 4   # the previous job is stale: abort its queued work

ALGO_KAWPOW, ALGO_EQUIHASH, ALGO_X16R, ALGO_X16RV2 = 0, 1, 2, 3
ALGO_NAMES = ("kawpow", "equihash", "x16r", "x16rv2")

EPOCH_PREBUILD_WINDOW = 120  # blocks before an epoch boundary at which the next DAG is prebuilt
LEGACY_WINDOW = 1 << 16      # nNonce values per host X16R window
LEGACY_GPU_WINDOW = 1 << 20  # nNonce values per GPU X16R window (~0.6 ms at 1.9 M hashes/s)
EQ_SOLUTION_PREFIX = b"\xfd\x40\x05"  # CompactSize(1344) in front of the packed solution


@dataclass(frozen=True)
class Work:
    header: bytes = bytes(80)
    boundary: bytes = bytes(32)      # share/block target, big-endian
    height: int = 0
    job_id: int = 0
    nonce_base: int = 0
    flags: int = FLAG_IDLE
    algo: int = ALGO_KAWPOW

    def __post_init__(self):
        if len(self.header) != 80:
            object.__setattr__(self, "header", bytes(self.header)[:80].ljust(80, b"\0"))

    @property
    def header_hash(self) -> bytes:
        """KawPow header hash (progpow storage order)."""
        return self.header[:32]

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
        return struct.pack(WORK_FMT, self.header, self.boundary, self.height, self.algo, self.job_id,
                           self.nonce_base, self.flags)

    @classmethod
    def unpack(cls, raw: bytes) -> "Work":
        hdr, b, height, algo, job, base, flags = struct.unpack(WORK_FMT, raw)
        return cls(hdr, b, height, job, base, flags, algo)

    def target64(self) -> int:
        """Upper 64 bits of the boundary: the kernel's prefix test never rejects a hash the full
        256-bit compare would accept."""
        return int.from_bytes(self.boundary[:8], "big")

    def target(self) -> int:
        return int.from_bytes(self.boundary, "big")


def equihash_nonce256(nonce: int) -> bytes:
    """The nonce256 a window's 64-bit nonce stands for (the rest of the space is left unused)."""
    return struct.pack("<Q", nonce & 0xFFFFFFFFFFFFFFFF) + bytes(24)


def equihash_block_hash(prefix80: bytes, nonce: int, solution: bytes) -> bytes:
    """SHA256d of the serialized extended header (storage order, as uint256): the Equihash
    extension's block hash (csrc/chain/primitives.cpp BlockHeader::equihash_hash)."""
    ser = prefix80 + equihash_nonce256(nonce) + EQ_SOLUTION_PREFIX + solution
    return hashlib.sha256(hashlib.sha256(ser).digest()).digest()


@dataclass
class EquihashShare:
    nonce: int           # the 64-bit nonce of equihash_nonce256
    solution: bytes      # 1344-byte packed solution
    block_hash: bytes    # SHA256d(header), storage order

    def nonce256(self) -> bytes:
        return equihash_nonce256(self.nonce)


@dataclass
class LegacyShare:
    nonce: int           # 32-bit nNonce
    block_hash: bytes    # X16R / X16RV2 hash, storage order


@dataclass
class SlotResult:
    """One finished window: the shares that pass the full 256-bit boundary and the work that was
    actually done (nonces hashed; Equihash: solutions found). An aborted window counts only the
    workgroups that ran; `aborted` is the number that did not."""
    job_id: int
    start: int
    count: int
    hashes: int
    shares: list = field(default_factory=list)
    device_ms: float = 0.0
    aborted: int = 0
    algo: int = ALGO_KAWPOW
    end_ms: float = 0.0  # device clock: the window's end, ms after the device's first window began


class DeviceHung(RuntimeError):
    """A window did not finish within the watchdog limit."""


class DeviceFault(RuntimeError):
    """A window failed on the device (a kernel error, a lost device, an injected fault)."""


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
        self.dag_build_s: dict[int, float] = {}
        nbytes = self.h.sizeof_results()
        with torch.cuda.device(self.device):
            # one stream per slot: the queued window starts on the CUs the running one's last
            # workgroups leave idle instead of waiting for its whole grid to drain (the tail of a
            # 2^25-nonce window is ~0.8 % of it; +0.3 % against one stream, profiles/README r4f)
            self.stream = torch.cuda.Stream(device=self.device)
            self.slot_streams = [self.stream, torch.cuda.Stream(device=self.device)]
            self.side = torch.cuda.Stream(device=self.device)  # next-epoch DAG builds
            self.rings = [torch.zeros(nbytes // 4, dtype=torch.int32, device=self.device) for _ in range(2)]
            self.host = [torch.zeros(nbytes // 4, dtype=torch.int32).pin_memory() for _ in range(2)]
            self.events = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            self.starts = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        self.meta: list[tuple | None] = [None, None]
        self.anchor = None  # timing event before the first window: SlotResult.end_ms is relative to it
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
        t0 = time.perf_counter()
        with torch.cuda.device(self.device):
            e = DeviceEpoch(epoch, device=self.device, world_size=ws)
            with torch.cuda.stream(stream or self.stream):
                if self.collective_dag:
                    pdag.build_dag(e)
                else:
                    e.build()
        self.dag_build_s[epoch] = time.perf_counter() - t0  # host-side issue time; completion below
        return e

    def epoch_ready(self, epoch: int) -> bool:
        return epoch in self.epochs

    def resident_epochs(self) -> list[int]:
        return sorted(self.epochs)

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
        t0 = time.perf_counter()
        if epoch in self.pending_build:
            e, ev = self.pending_build.pop(epoch)
            for st in self.slot_streams:
                st.wait_event(ev)  # search kernels after the build, without a host sync
        else:
            e = self._build_epoch(epoch)
        with torch.cuda.device(self.device):
            for st in self.slot_streams:
                st.synchronize()
            if not e.l1_matches():
                raise RuntimeError(f"gpu{self.device}: epoch {epoch} DAG failed its L1 self-check")
        self.dag_build_s[epoch] = self.dag_build_s.get(epoch, 0.0) + time.perf_counter() - t0
        from ..ops import verify as V

        V.share_epoch(self.device, epoch, e)  # header batches of this epoch verify against it too
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

    def window_for(self, work: Work, window: int) -> int:
        b = self.block_for(work.height)
        return max(b, window // b * b)

    # ------------------------------------------------------------------ the two slots
    def submit(self, slot: int, work: Work, start: int, count: int) -> None:
        torch = self.torch
        s = self.searcher(work.height)
        b = s.block
        count = max(b, count // b * b)
        st = self.slot_streams[slot]
        with torch.cuda.device(self.device), torch.cuda.stream(st):
            ring = self.rings[slot]
            ring[:4].zero_()
            if self.anchor is None:
                self.anchor = torch.cuda.Event(enable_timing=True)
                self.anchor.record(st)
            self.starts[slot].record(st)
            s.launch(work.header_hash, start, count, work.target64(), stream=int(st.cuda_stream),
                     results=ring, gen_word=self.gen_ptr, generation=self.generation)
            self.host[slot].copy_(ring, non_blocking=True)
            self.events[slot].record(st)
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
        return SlotResult(work.job_id, start, count, hashes, shares, self.starts[slot].elapsed_time(ev), skipped,
                          ALGO_KAWPOW, self.anchor.elapsed_time(ev))

    def abort(self) -> None:
        """Make every queued or running window stale (its remaining workgroups exit at start)."""
        self.generation = (self.generation + 1) & 0xFFFFFFFF
        self.h.host_word_store(self.gen_ptr, 0, self.generation)

    def synchronize(self) -> None:
        for st in self.slot_streams:
            st.synchronize()


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

    def window_for(self, work: Work, window: int) -> int:
        return max(1, min(int(window), self.max_window))

    def epoch_ready(self, epoch: int) -> bool:
        return True

    def resident_epochs(self) -> list[int]:
        return []

    def prebuild(self, epoch: int) -> None:
        _core.get_epoch_context(epoch)

    def submit(self, slot: int, work: Work, start: int, count: int) -> None:
        self.meta[slot] = (work, start, min(count, self.max_window), self.generation)

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        from ..ops.kawpow import Share

        work, start, count, gen = self.meta[slot]
        self.meta[slot] = None
        if gen != self.generation:  # aborted before it ran
            return SlotResult(work.job_id, start, count, 0, [], 0.0, 1, ALGO_KAWPOW)
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


class LegacyHostDevice:
    """X16R / X16RV2 templates (before the KawPow activation; the regtest default): the 32-bit
    nNonce scanned on the host cores by the native multi-threaded search (csrc/pow/x16r.cpp,
    `_core.x16r_search`), first hit of each window — generateBlocks' loop (src/rpc/mining.cpp:
    141-149) in windows. The 32-bit space is split 2^28 per rank (`start` wraps inside it)."""

    name = "host-x16r"
    device = -1

    def __init__(self):
        self.meta: list[tuple | None] = [None, None]
        self.generation = 0

    def window_for(self, work: Work, window: int) -> int:
        return LEGACY_WINDOW

    def submit(self, slot: int, work: Work, start: int, count: int) -> None:
        self.meta[slot] = (work, start & 0xFFFFFFFF, count, self.generation)

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        work, start, count, gen = self.meta[slot]
        self.meta[slot] = None
        if gen != self.generation:
            return SlotResult(work.job_id, start, count, 0, [], 0.0, 1, work.algo)
        count = min(count, (1 << 32) - start)
        t0 = time.perf_counter()
        target_le = work.boundary[::-1]
        res, hashes = _core.x16r_search(work.header, work.algo == ALGO_X16RV2, target_le, start, count)
        dt = (time.perf_counter() - t0) * 1e3
        shares = [LegacyShare(int(res[0]), bytes(res[1]))] if res is not None else []
        return SlotResult(work.job_id, start, count, int(hashes), shares, dt, 0, work.algo)

    def abort(self) -> None:
        self.generation += 1

    def synchronize(self) -> None:
        pass

    def close(self) -> None:
        pass


class LegacyGpuDevice(LegacyHostDevice):
    """The same X16R / X16RV2 windows on this rank's GPU (ops/x16r.X16rSearcher: every nonce of a
    window runs the same 16 slots, one launch per step, the lowest hit kept on the device)."""

    name = "gpu-x16r"

    def __init__(self, device: int = 0, window: int = LEGACY_GPU_WINDOW):
        super().__init__()
        self.device = int(device)
        self._window = int(window)
        self._searcher = None

    def window_for(self, work: Work, window: int) -> int:
        return self._window

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        work, start, count, gen = self.meta[slot]
        self.meta[slot] = None
        if gen != self.generation:
            return SlotResult(work.job_id, start, count, 0, [], 0.0, 1, work.algo)
        count = min(count, (1 << 32) - start)
        if self._searcher is None:
            from ..ops.x16r import X16rSearcher

            self._searcher = X16rSearcher(self.device, window=self._window)
        t0 = time.perf_counter()
        res, hashes = self._searcher.search(work.header, work.algo == ALGO_X16RV2, work.boundary[::-1], start, count)
        dt = (time.perf_counter() - t0) * 1e3
        shares = [LegacyShare(int(res[0]), bytes(res[1]))] if res is not None else []
        return SlotResult(work.job_id, start, count, int(hashes), shares, dt, 0, work.algo)


class RankDevice:
    """Everything one rank mines with, behind the two-slot protocol: the KawPow device (GPU or host),
    the Equihash device (made on first use: GPU solver or host golden solver) and the host X16R
    search. Each slot goes to the device of its work's algorithm, so a chain crossing an activation
    time switches algorithms between two windows with no change to the loop."""

    def __init__(self, kawpow, equihash=None, legacy=None, equihash_factory=None):
        self.kawpow = kawpow
        self._equihash = equihash
        self._eq_factory = equihash_factory
        self.legacy = legacy if legacy is not None else LegacyHostDevice()
        self.slot_dev: list[object | None] = [None, None]
        self.name = getattr(kawpow, "name", "dev")
        self.device = getattr(kawpow, "device", -1)

    @property
    def collective_dag(self) -> bool:
        return getattr(self.kawpow, "collective_dag", False)

    @property
    def equihash(self):
        if self._equihash is None:
            if self._eq_factory is None:
                from .equihash_search import EquihashCpuDevice

                self._equihash = EquihashCpuDevice()
            else:
                self._equihash = self._eq_factory()
        return self._equihash

    def dev_for(self, work: Work):
        if work.algo == ALGO_KAWPOW:
            return self.kawpow
        if work.algo == ALGO_EQUIHASH:
            return self.equihash
        return self.legacy

    def window_for(self, work: Work, window: int) -> int:
        return self.dev_for(work).window_for(work, window)

    def block_for(self, height: int) -> int:
        return self.kawpow.block_for(height)

    def epoch_ready(self, epoch: int) -> bool:
        return self.kawpow.epoch_ready(epoch)

    def resident_epochs(self) -> list[int]:
        return self.kawpow.resident_epochs() if hasattr(self.kawpow, "resident_epochs") else []

    def prebuild(self, epoch: int) -> None:
        self.kawpow.prebuild(epoch)

    def submit(self, slot: int, work: Work, start: int, count: int) -> None:
        d = self.dev_for(work)
        self.slot_dev[slot] = d
        d.submit(slot, work, start, count)

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        d, self.slot_dev[slot] = self.slot_dev[slot], None
        return d.wait(slot, timeout_s)

    def abort(self) -> None:
        for d in (self.kawpow, self._equihash, self.legacy):
            if d is not None:
                d.abort()

    def synchronize(self) -> None:
        for d in (self.kawpow, self._equihash):
            if d is not None:
                d.synchronize()

    def close(self) -> None:
        for d in (self.kawpow, self._equihash, self.legacy):
            if d is not None and hasattr(d, "close"):
                d.close()


def as_rank_device(dev) -> RankDevice:
    """A bare device becomes a rank's device for its own algorithm: an Equihash device serves the
    Equihash windows (a KawPow or X16R packet would find no device of its kind and fail), any
    other device the KawPow ones."""
    if isinstance(dev, (RankDevice, FaultInjectingDevice, HangingDevice)):
        return dev
    if getattr(dev, "algo", None) == ALGO_EQUIHASH:
        return RankDevice(_NoKawpow(dev), equihash=dev)
    return RankDevice(dev)


class _NoKawpow:
    """The KawPow slot of a rank that only has an Equihash device (bench.py's Equihash loop)."""

    def __init__(self, eq):
        self.name, self.device = eq.name, eq.device

    def window_for(self, work, window):
        raise DeviceFault("this rank has no KawPow device")

    submit = block_for = window_for

    def epoch_ready(self, epoch: int) -> bool:
        return True

    def resident_epochs(self) -> list[int]:
        return []

    def prebuild(self, epoch: int) -> None:
        pass

    def abort(self) -> None:
        pass

    def synchronize(self) -> None:
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


class _Wrapper:
    def __init__(self, inner):
        self.inner = inner

    def __getattr__(self, name):
        return getattr(self.inner, name)


class FaultInjectingDevice(_Wrapper):
    """-gpufailrate / -dropshare (SURVEY §5 fault injection; never on by default): each window fails
    with probability `fail_rate` (wait() raises DeviceFault after the window ran, as a device error
    surfaces), and each share is silently lost with probability `drop_rate` (a share lost between
    device and host). Wraps any device of the two-slot protocol."""

    def __init__(self, inner, fail_rate: float = 0.0, drop_rate: float = 0.0, seed: int | None = None):
        import random

        super().__init__(inner)
        self.fail_rate, self.drop_rate = float(fail_rate), float(drop_rate)
        self.rng = random.Random(seed)
        self.dropped = 0
        self.faults = 0

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        res = self.inner.wait(slot, timeout_s)
        if self.fail_rate and self.rng.random() < self.fail_rate:
            self.faults += 1
            raise DeviceFault(f"injected device fault on {getattr(self.inner, 'name', 'dev')}")
        if self.drop_rate and res.shares:
            kept = [s for s in res.shares if self.rng.random() >= self.drop_rate]
            self.dropped += len(res.shares) - len(kept)
            res.shares = kept
        return res


class HangingDevice(_Wrapper):
    """Fault injection (tests, `NODEXA_MINER_HANG_AFTER`): behaves like `inner` for `after` windows,
    then every window hangs — wait() blocks until the watchdog limit and raises DeviceHung, which is
    what a GPU whose kernel never returns looks like to the mining loop."""

    def __init__(self, inner, after: int):
        super().__init__(inner)
        self.after = int(after)
        self.waits = 0

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        self.waits += 1
        if self.waits <= self.after:
            return self.inner.wait(slot, timeout_s)
        time.sleep(timeout_s if timeout_s is not None else 1e9)
        raise DeviceHung(f"{getattr(self.inner, 'name', 'dev')}: injected hang")
