"""The node's KawPow miner: one process per GPU, nonce-space data parallelism over RCCL.

Reference: GenerateClores / CloreMiner (src/miner.cpp:566-759) run N host threads, each with its
own template and a 32-bit nonce scan, and getmininginfo reports their nHashesPerSec
(src/rpc/mining.cpp:209-250). Here every GPU is a rank of one torch.distributed world (backend
"nccl" = RCCL over xGMI on the MI355X node; "gloo" for CPU rehearsals) and all ranks run the
same loop, `MiningService.step`:

  1. queue the next 2^25-nonce window on this rank's device and take the previous window's
     result (miner/search.SearchPipeline: the GPU never waits for the host);
  2. all-gather every rank's share record (fixed 1176-byte slot: job, hashes, up to 16 shares);
  3. all-reduce the step's hash counters (and the next-epoch readiness votes);
  4. rank 0 (the node: chain state, RPC) fully re-hashes shares in light mode, builds the block
     of the share's job and runs ProcessNewBlock; then it decides the next work packet;
  5. broadcast the 96-byte work packet from rank 0; a new job with FLAG_CLEAN makes every rank
     abort its queued window of the stale job on the device.

Nonce partition: rank r of n searches job-local windows from nonce_base + (r << 56), so ranks
never overlap and a job change (new extranonce -> new header hash) restarts every cursor.
DAGs are built sharded over the ranks and all-gathered (parallel/dag.py); the next epoch's DAG is
prebuilt on a side stream once every rank reports its light cache ready (an all-reduced vote, so
the collective build starts on the same step everywhere).

Failure handling: a rank whose window outlives the watchdog exits with
EXIT_DEVICE_HUNG (a fresh process on restart, never a re-exec). Survivors see their next
collective fail or time out, register in the rendezvous store under a new membership epoch, wait
out a grace period, rebuild the group over the ranks that registered (parallel/world.shrink) and
carry on; rank 0 then issues a clean job so the nonce space is re-partitioned over the new ranks.
"""
from __future__ import annotations

import datetime
import os
import struct
import sys
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field

from .. import core
from ..utils import log
from .search import (EPOCH_PREBUILD_WINDOW, FLAG_CLEAN, FLAG_IDLE, FLAG_STOP, WORK_SIZE, DeviceHung,
                     SearchPipeline, SlotResult, Work)

_core = core()

EXIT_DEVICE_HUNG = 75
MAX_SHARES_PER_STEP = 16
_REC_HEAD = struct.Struct("<QQII")           # job_id, hashes, nshares, flags
_REC_SHARE = struct.Struct("<Q32s32s")        # nonce, mix, final
RECORD_SIZE = _REC_HEAD.size + MAX_SHARES_PER_STEP * _REC_SHARE.size  # 1176


class CollectiveError(RuntimeError):
    """A collective of the mining loop failed or timed out (a peer rank is gone or hung)."""


def pack_record(res: SlotResult | None) -> bytes:
    if res is None:
        return bytes(RECORD_SIZE)
    shares = res.shares[:MAX_SHARES_PER_STEP]
    out = bytearray(RECORD_SIZE)
    _REC_HEAD.pack_into(out, 0, res.job_id, res.hashes, len(shares), 1)
    for i, s in enumerate(shares):
        _REC_SHARE.pack_into(out, _REC_HEAD.size + i * _REC_SHARE.size, s.nonce, s.mix_hash, s.final_hash)
    return bytes(out)


def unpack_record(raw: bytes) -> tuple[int, int, list]:
    from ..ops.kawpow import Share

    job, hashes, n, _flags = _REC_HEAD.unpack_from(raw, 0)
    shares = [Share(*_REC_SHARE.unpack_from(raw, _REC_HEAD.size + i * _REC_SHARE.size))
              for i in range(min(n, MAX_SHARES_PER_STEP))]
    return job, hashes, shares


class Comm:
    """The loop's collectives on the current world group, each bounded by a timeout.

    RCCL: tensors live on the GPU and the collectives are issued from a stream of their own, so
    they never queue behind the search kernel that is running on the search stream. gloo: host
    tensors. A single rank needs no collective at all."""

    def __init__(self, timeout_s: float):
        import torch

        from ..parallel import world as W

        self.torch = torch
        self.W = W
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.rebind()

    def rebind(self) -> None:
        """Bind to the current world. The loop gets a communicator of its own (not the default
        group), so a failed one can be aborted (RCCL) and replaced without touching the default
        group or its rendezvous store."""
        torch, dist = self.torch, self.W.dist
        self.w = self.W.get()
        self.gpu = self.w.backend == "nccl"
        self.stream = torch.cuda.Stream(device=self.w.device) if self.gpu else None
        self.group = self.w.group
        if self.w.distributed and self.group is None:
            self.group = dist.new_group(ranks=list(range(self.w.world_size)), timeout=self.timeout)

    def abort(self) -> None:
        """Tear down the loop's communicator after a failure: RCCL kernels still waiting for a dead
        peer are cancelled (ncclCommAbort); gloo needs nothing (its ops already raised)."""
        if self.gpu and self.group is not None:
            try:
                self.W.dist.distributed_c10d._abort_process_group(self.group)
            except Exception as e:  # noqa: BLE001 — best effort; the survivors re-form regardless
                log.log_printf(f"miner: aborting the failed communicator: {e}")

    def _wait(self, work, what: str) -> None:
        try:
            ok = work.wait(timeout=self.timeout)
        except Exception as e:  # noqa: BLE001 — gloo raises on a closed peer, RCCL on timeout
            raise CollectiveError(f"{what}: {e}") from e
        if ok is False:
            raise CollectiveError(f"{what}: timed out")

    def _run(self, fn, what: str):
        torch = self.torch
        if self.gpu:
            with torch.cuda.device(self.w.device), torch.cuda.stream(self.stream):
                out = fn()
                self.stream.synchronize()
                return out
        return fn()

    def broadcast(self, payload: bytes | None, size: int) -> bytes:
        if not self.w.distributed:
            return payload
        torch, dist = self.torch, self.W.dist

        def go():
            t = torch.zeros(size, dtype=torch.uint8)
            if self.w.rank == 0:
                t.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
            if self.gpu:
                t = t.to(self.w.device, non_blocking=True)
            self._wait(dist.broadcast(t, src=self.w.global_rank(0), group=self.group, async_op=True), "broadcast")
            return bytes(t.cpu().numpy().tobytes())

        return self._run(go, "broadcast")

    def all_gather(self, record: bytes) -> list[bytes]:
        if not self.w.distributed:
            return [record]
        torch, dist = self.torch, self.W.dist
        n, ws = len(record), self.w.world_size

        def go():
            mine = torch.frombuffer(bytearray(record), dtype=torch.uint8)
            if self.gpu:
                mine = mine.to(self.w.device, non_blocking=True)
                out = torch.empty(ws * n, dtype=torch.uint8, device=self.w.device)
                self._wait(dist.all_gather_into_tensor(out, mine, group=self.group, async_op=True), "all_gather")
            else:
                out = torch.empty(ws * n, dtype=torch.uint8)
                parts = list(out.view(ws, n).unbind(0))
                self._wait(dist.all_gather(parts, mine, group=self.group, async_op=True), "all_gather")
            raw = bytes(out.cpu().numpy().tobytes())
            return [raw[i * n:(i + 1) * n] for i in range(ws)]

        return self._run(go, "all_gather")

    def all_reduce_sum(self, vals: list[int]) -> list[int]:
        if not self.w.distributed:
            return list(vals)
        torch, dist = self.torch, self.W.dist

        def go():
            t = torch.tensor(vals, dtype=torch.int64)
            if self.gpu:
                t = t.to(self.w.device, non_blocking=True)
            self._wait(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True), "all_reduce")
            return [int(x) for x in t.cpu().tolist()]

        return self._run(go, "all_reduce")


class RateMeter:
    """Hashes per second over a sliding window (getmininginfo.hashespersec)."""

    def __init__(self, window_s: float = 8.0):
        self.window_s = window_s
        self.samples: list[tuple[float, int]] = []
        self.lock = threading.Lock()

    def add(self, hashes: int, now: float | None = None) -> None:
        now = time.monotonic() if now is None else now
        with self.lock:
            self.samples.append((now, hashes))
            while len(self.samples) > 2 and now - self.samples[1][0] > self.window_s:
                self.samples.pop(0)

    def rate(self) -> float:
        with self.lock:
            if len(self.samples) < 2:
                return 0.0
            dt = self.samples[-1][0] - self.samples[0][0]
            return sum(h for _, h in self.samples[1:]) / dt if dt > 0 else 0.0


@dataclass
class MiningRequest:
    """generate / setgenerate on rank 0: mine with `script` until `blocks` are found (None =
    until stopped) or `max_tries` hashes are spent."""
    script: bytes
    blocks: int | None = None
    max_tries: int | None = None
    found: list = field(default_factory=list)
    tries: int = 0
    done: threading.Event = field(default_factory=threading.Event)
    error: str | None = None


@dataclass
class Job:
    job_id: int
    block: object
    height: int
    header_hash: bytes
    boundary: bytes
    prev: bytes
    tx_updated: int
    created: float
    script: bytes


class ChainLeader:
    """Rank 0's side of the loop: templates -> work packets, shares -> blocks.

    Templates come from BlockAssembler (src/miner.cpp:123-256) with IncrementExtraNonce
    (:508-525) per job; a job is replaced when the tip moves, when the pool changed and the job is
    older than `refresh_s` (the reference's 60 s mempool check, src/miner.cpp:700-705), or when
    the world was re-partitioned. Every share is re-hashed in full (light mode) before its block is
    built; only shares of a job whose parent is still the tip are submitted (the reference's
    "generated block is stale" check, ProcessBlockFound)."""

    def __init__(self, state, *, refresh_s: float = 10.0, target_bits: int = 0, on_block=None):
        from .assembler import ExtraNonce

        self.state = state
        self.refresh_s = float(refresh_s)
        self.miner_target = (1 << (256 - int(target_bits))) - 1 if target_bits else None
        self.on_block = on_block
        self.jobs: OrderedDict[int, Job] = OrderedDict()
        self.job_seq = 0
        self.extranonce = ExtraNonce()
        self.request: MiningRequest | None = None
        self.lock = threading.Lock()
        self.force_new = False
        self.stopping = False
        self.stats = {"shares": 0, "stale_shares": 0, "bad_shares": 0, "blocks": 0, "rejected": 0}

    # ---------------------------------------------------------------- called from RPC threads
    def mine(self, script: bytes, blocks: int | None = None, max_tries: int | None = None) -> MiningRequest:
        req = MiningRequest(script, blocks, max_tries)
        with self.lock:
            old, self.request = self.request, req
            self.force_new = True
        if old is not None and not old.done.is_set():
            old.error = old.error or "superseded"
            old.done.set()
        return req

    def stop_mining(self) -> None:
        with self.lock:
            req, self.request = self.request, None
        if req is not None:
            req.done.set()

    def shutdown(self) -> None:
        self.stop_mining()
        self.stopping = True

    # ---------------------------------------------------------------- called from the loop thread
    def next_work(self, repartitioned: bool = False) -> Work:
        from ..chain.header import to_progpow
        from .assembler import BlockAssembler

        if self.stopping:
            return Work(flags=FLAG_STOP)
        with self.lock:
            req = self.request
            force = self.force_new or repartitioned
            self.force_new = False
        if req is None or req.done.is_set():
            return Work(flags=FLAG_IDLE)
        st = self.state
        tip = st.tip()
        cur = next(reversed(self.jobs.values())) if self.jobs else None
        stale = (cur is None or force or cur.prev != tip.hash or cur.script != req.script
                 or (st.transactions_updated != cur.tx_updated and time.time() - cur.created > self.refresh_s))
        if not stale:
            return Work(cur.header_hash, cur.boundary, cur.height, cur.job_id, 0, 0)
        tpl = BlockAssembler(st).create_new_block(req.script)
        blk = tpl.block
        if blk.header.time < st.params.kawpow_activation_time:
            req.error = "template is before the KawPow activation time (X16R/X16RV2 is mined on the host)"
            req.done.set()
            return Work(flags=FLAG_IDLE)
        self.extranonce.increment(blk, tpl.height)
        hdr = blk.header
        target = tpl.target if self.miner_target is None else min(tpl.target, self.miner_target)
        self.job_seq += 1
        job = Job(self.job_seq, blk, tpl.height, to_progpow(hdr.kawpow_header_hash()), target.to_bytes(32, "big"),
                  hdr.prev, st.transactions_updated, time.time(), req.script)
        self.jobs[job.job_id] = job
        while len(self.jobs) > 8:
            self.jobs.popitem(last=False)
        return Work(job.header_hash, job.boundary, job.height, job.job_id, 0, FLAG_CLEAN)

    def on_results(self, records: list[tuple[int, int, list]]) -> None:
        from ..chain.header import from_progpow

        req = self.request
        hashes = sum(h for _, h, _ in records)
        if req is None:
            return
        req.tries += hashes
        st = self.state
        act = st.params.kawpow_activation_time
        for job_id, _h, shares in records:
            for sh in shares:
                if req.done.is_set():
                    break
                self.stats["shares"] += 1
                job = self.jobs.get(job_id)
                if job is None or job.prev != st.tip().hash:
                    self.stats["stale_shares"] += 1
                    continue
                if not sh.verify_full(job.height, job.header_hash, job.boundary):
                    self.stats["bad_shares"] += 1
                    log.log_printf(f"miner: share nonce {sh.nonce:#x} of job {job_id} failed full re-hash; dropped")
                    continue
                blk = _core.Block.deserialize(job.block.serialize(act), act)
                hdr = blk.header
                hdr.nonce64 = sh.nonce
                hdr.mix_hash = from_progpow(sh.mix_hash)
                blk.header = hdr
                res = st.process_new_block(blk)
                if not res.ok:
                    self.stats["rejected"] += 1
                    log.log_printf(f"miner: block of job {job_id} rejected: {res.reject}")
                    continue
                bh = st.block_hash(hdr)
                self.stats["blocks"] += 1
                req.found.append(_core.u256_hex(bh))
                st._emit("block_found", bh)
                if self.on_block is not None:
                    self.on_block(blk)
                self.force_new = True
                if req.blocks is not None and len(req.found) >= req.blocks:
                    req.done.set()
                break  # one block per job: the next one builds on it
        if req.max_tries is not None and req.tries >= req.max_tries:
            req.done.set()


class BenchLeader:
    """A fixed synthetic job (bench.py): the same loop, no chain. Shares are kept for the full
    re-hash check after the timed region."""

    def __init__(self, work: Work, keep: int = 64):
        self.work = Work(work.header_hash, work.boundary, work.height, work.job_id or 1, work.nonce_base, 0)
        self.first = True
        self.keep = keep
        self.shares: list = []
        self.stopping = False

    def next_work(self, repartitioned: bool = False) -> Work:
        if self.stopping:
            return Work(flags=FLAG_STOP)
        if self.first or repartitioned:
            self.first = False
            w = self.work
            return Work(w.header_hash, w.boundary, w.height, w.job_id, w.nonce_base, FLAG_CLEAN)
        return self.work

    def on_results(self, records) -> None:
        for _job, _h, shares in records:
            if len(self.shares) < self.keep:
                self.shares.extend(shares[:self.keep - len(self.shares)])

    def shutdown(self) -> None:
        self.stopping = True


class MiningService:
    """The per-rank mining loop (see the module docstring). Rank 0 passes a leader."""

    def __init__(self, device, leader=None, *, window: int = 1 << 25, watchdog_s: float = 120.0,
                 collective_timeout_s: float = 60.0, grace_s: float | None = None, idle_sleep_s: float = 0.02,
                 record_windows: bool = False):
        from ..parallel import world as W

        self.W = W
        self.dev = device
        self.leader = leader
        self.window = int(window)
        self.pipe = SearchPipeline(device, watchdog_s)
        self.comm = Comm(collective_timeout_s)
        self.collective_timeout_s = float(collective_timeout_s)
        self.grace_s = float(grace_s) if grace_s is not None else 2 * self.collective_timeout_s + 1
        self.idle_sleep_s = float(idle_sleep_s)
        self.work = Work()
        self.cursor = 0
        self.rate = RateMeter()
        self.hashes_total = 0
        self.rank_hashes: dict[int, int] = {}
        self.steps = 0
        self.membership = 0
        self.repartitioned = False
        self.windows: list[tuple[int, int, int]] | None = [] if record_windows else None
        self._light_thread: threading.Thread | None = None
        self._thread: threading.Thread | None = None
        self.error: BaseException | None = None
        self.last_step_ms = 0.0

    @property
    def rank(self) -> int:
        return self.comm.w.rank

    @property
    def world_size(self) -> int:
        return self.comm.w.world_size

    def hashrate(self) -> float:
        return self.rate.rate()

    # ---------------------------------------------------------------- one step
    def _next_epoch_vote(self) -> int:
        """1 when this rank has the next epoch's light cache (prebuild window only)."""
        w = self.work
        if w.idle or w.height % _core.EPOCH_LENGTH < _core.EPOCH_LENGTH - EPOCH_PREBUILD_WINDOW:
            return 0
        nxt = w.epoch + 1
        if self.dev.epoch_ready(nxt):
            return 0
        t = self._light_thread
        if t is None:
            t = threading.Thread(target=_core.get_epoch_context, args=(nxt,), name=f"light-{nxt}", daemon=True)
            self._light_thread = t
            t.start()
        if t.is_alive():
            return 0
        return 1

    def step(self) -> bool:
        """One iteration of the loop on this rank; False once a stop packet has been processed."""
        t0 = time.perf_counter()
        w = self.work
        if w.idle:
            res = self.pipe.drain()
            if res is None:
                time.sleep(self.idle_sleep_s)
        else:
            start = w.nonce_base + (self.rank << 56) + self.cursor
            block = self.dev.block_for(w.height)
            count = max(block, self.window // block * block)
            if self.windows is not None:
                self.windows.append((w.job_id, start, count))
            res = self.pipe.step(w, start, count)
            self.cursor += count
        vote = self._next_epoch_vote()
        gathered = self.comm.all_gather(pack_record(res))
        sums = self.comm.all_reduce_sum([res.hashes if res is not None else 0, vote])
        self.hashes_total += sums[0]
        self.rate.add(sums[0])
        if vote and sums[1] == self.world_size:
            # every rank holds the light cache: all start the (collective) build on this step
            self.dev.prebuild(w.epoch + 1)
            self._light_thread = None
        payload = None
        if self.leader is not None:
            records = [unpack_record(r) for r in gathered]
            for i, (_j, h, _s) in enumerate(records):
                self.rank_hashes[i] = self.rank_hashes.get(i, 0) + h
            self.leader.on_results(records)
            payload = self.leader.next_work(self.repartitioned).pack()
            self.repartitioned = False
        new = Work.unpack(self.comm.broadcast(payload, WORK_SIZE))
        if new.job_id != w.job_id:
            self.cursor = 0
        if new.flags & FLAG_CLEAN or new.idle:
            self.dev.abort()  # the window queued for the old job stops on the device
        self.work = new
        self.steps += 1
        self.last_step_ms = (time.perf_counter() - t0) * 1e3
        return not new.stop

    # ---------------------------------------------------------------- failures
    def recover(self, err: Exception) -> None:
        """Survivor side of a lost rank: membership by rendezvous-store registration, then a new
        group over the registered ranks. Raises if the leader (global rank 0) is among the lost."""
        import torch.distributed as dist

        W = self.W
        w = W.get()
        members = list(w.ranks or range(w.world_size))
        me = w.global_rank(w.rank)
        self.membership += 1
        store = dist.distributed_c10d._get_default_store()
        prefix = f"nodexa/miner/m{self.membership}/alive/"
        store.set(prefix + str(me), "1")
        log.log_printf(f"miner rank {me}: collective failed ({err}); membership round {self.membership}")
        deadline = time.monotonic() + self.grace_s
        alive = [me]
        while time.monotonic() < deadline:
            alive = [r for r in members if store.check([prefix + str(r)])]
            if len(alive) == len(members):
                break
            time.sleep(0.05)
        if members[0] not in alive:
            raise RuntimeError(f"miner leader (rank {members[0]}) is gone")
        try:
            self.pipe.drain()
        except DeviceHung:
            raise
        except Exception:  # noqa: BLE001 — the window of the broken step is discarded
            pass
        self.comm.abort()
        W.shrink(alive, timeout_s=int(max(1, self.collective_timeout_s)))
        self.comm.rebind()
        self.work = Work()
        self.cursor = 0
        self.repartitioned = True
        log.log_printf(f"miner rank {me}: continuing as rank {self.rank} of {self.world_size} (ranks {alive})")

    def run(self, stop: threading.Event | None = None) -> None:
        """Loop until a stop packet (followers) or `stop` is set and the stop packet went out (leader)."""
        while True:
            if stop is not None and stop.is_set() and self.leader is not None:
                self.leader.shutdown()
            try:
                if not self.step():
                    break
            except CollectiveError as e:
                self.recover(e)
        try:
            self.pipe.drain()
        except Exception:  # noqa: BLE001
            pass

    def start(self) -> "MiningService":
        """Run the loop on a background thread (rank 0 inside the node)."""
        self._stop = threading.Event()

        def go():
            try:
                self.run(self._stop)
            except BaseException as e:  # noqa: BLE001 — surfaced through getmininginfo / logs
                self.error = e
                log.log_printf(f"miner loop stopped: {type(e).__name__}: {e}")
                if self.leader is not None and getattr(self.leader, "request", None) is not None:
                    self.leader.request.error = str(e)
                    self.leader.request.done.set()

        self._thread = threading.Thread(target=go, name="miner-service", daemon=True)
        self._thread.start()
        return self

    def stop(self, timeout: float = 30.0) -> None:
        if self._thread is None:
            return
        self._stop.set()
        self._thread.join(timeout)
        self._thread = None


# -------------------------------------------------------------------- follower processes
def spawn_followers(gpus: list[int], port: int, cpu: bool = False, extra_env: dict | None = None) -> list:
    """Start ranks 1..n-1 of the miner world as child processes (before this process touches a GPU;
    they are started, never exec'd over a GPU process). Rank r drives gpus[r]."""
    import subprocess

    procs = []
    n = len(gpus)
    for r in range(1, n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_RANK": str(r), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "NODEXA_MINER_DEVICE": str(gpus[r]),
                    "NODEXA_MINER_CPU": "1" if cpu else "0"})
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, "-m", "nodexa_chain_core_amd.miner.service"], env=env))
    return procs


def follower_main() -> int:
    """Entry point of ranks >= 1 (spawned by the node or launched by torchrun)."""
    from ..parallel import world as W

    cpu = os.environ.get("NODEXA_MINER_CPU", "0") == "1"
    dev_index = os.environ.get("NODEXA_MINER_DEVICE")
    timeout = float(os.environ.get("NODEXA_MINER_COLLECTIVE_TIMEOUT", "60"))
    watchdog = float(os.environ.get("NODEXA_MINER_WATCHDOG", "120"))
    window = int(os.environ.get("NODEXA_MINER_WINDOW", str(1 << 25)))
    W.init(use_gpu=not cpu, device_index=None if dev_index is None else int(dev_index),
           timeout_s=int(max(timeout, 10)), elastic=True)
    if cpu:
        from .search import CpuSearchDevice

        dev = CpuSearchDevice(max_window=window)
    else:
        from .search import GpuSearchDevice

        dev = GpuSearchDevice(W.get().device.index, collective_dag=W.get().distributed)
    hang = int(os.environ.get("NODEXA_MINER_HANG_AFTER", "0"))
    if hang > 0:  # fault injection for the failure-handling tests
        from .search import HangingDevice

        dev = HangingDevice(dev, hang)
    wlog = os.environ.get("NODEXA_MINER_WINDOWS_LOG")
    svc = MiningService(dev, None, window=window, watchdog_s=watchdog, collective_timeout_s=timeout,
                        record_windows=bool(wlog))

    def dump():
        if wlog:
            import json

            with open(wlog, "w") as f:
                json.dump({"rank": svc.rank, "world_size": svc.world_size, "windows": svc.windows,
                           "steps": svc.steps, "hashes_total": svc.hashes_total}, f)

    try:
        svc.run()
    except DeviceHung as e:
        log.log_printf(f"miner rank {W.get().rank}: {e}; exiting so the survivors re-partition")
        dump()
        os._exit(EXIT_DEVICE_HUNG)
    except RuntimeError as e:
        log.log_printf(f"miner rank {W.get().rank}: {e}")
        dump()
        return 3
    dump()
    W.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(follower_main())
