"""The node's miner: one process per GPU, nonce-space data parallelism over RCCL.

Reference: GenerateClores / CloreMiner (src/miner.cpp:566-759) run N host threads, each with its
own template and a 32-bit nonce scan; generateBlocks (src/rpc/mining.cpp:117-173) is a second,
separate loop; getmininginfo reports nHashesPerSec (src/rpc/mining.cpp:209-250). Here there is
one loop for everything. Every GPU is a rank of one torch.distributed world (backend "nccl" =
RCCL over xGMI on the MI355X node; "gloo" for CPU rehearsals; a single CPU-only rank needs no
process group at all) and all ranks run the same step, `MiningService.step`:

  1. queue the next window on this rank's device and take the previous window's result
     (miner/search.SearchPipeline: the GPU never waits for the host). The work packet says which
     proof of work: KawPow (2^25-nonce GPU windows), Equihash(200,9) (16 solver instances per
     window) or X16R/X16RV2 (host windows of 2^16 nNonce values, before the KawPow activation);
  2. all-gather every rank's record (fixed 5592-byte slot: job, work done, shares, and the rank's
     own telemetry: device time, aborted workgroups, collective wait, failures, resident epochs,
     next-epoch readiness vote); every rank sums the work counters and votes from it;
  3. rank 0 (the node: chain state, RPC) checks shares again (KawPow: full light-mode re-hash;
     Equihash: the golden verifier; X16R: the block check), builds the block of the share's job
     and runs ProcessNewBlock; then it decides the next work packet;
  4. broadcast the 144-byte work packet from rank 0; a new job with FLAG_CLEAN makes every rank
     abort its queued window of the stale job on the device.

Nonce partition: rank r of n searches job-local windows from nonce_base + (r << 56) (X16R's 32-bit
nNonce: r << 28), so ranks never overlap and a job change (new extranonce -> new header) restarts
every cursor. DAGs are built sharded over the ranks and all-gathered (parallel/dag.py); the next
epoch's DAG is prebuilt on a side stream once every rank reports its light cache ready (a vote in
the gathered records, so the collective build starts on the same step everywhere). On RCCL the two
collectives run from a high-priority stream with persistent pinned/device buffers, so they never
queue behind a search window on a shared hardware queue.

Failure handling (the reference's miner just exits on errors, src/miner.cpp:716-725):
* a window that raises (a device fault; -gpufailrate injects them) counts a failure; after
  `max_failures` in a row the rank's device is evicted: a follower rank exits with
  EXIT_DEVICE_FAILED and the survivors re-form without it, rank 0 keeps leading without searching;
* a rank whose window outlives the watchdog exits with EXIT_DEVICE_HUNG (a fresh process on
  restart, never a re-exec). Survivors see their next collective fail or time out, register in the
  rendezvous store under a new membership epoch, wait out a grace period, rebuild the group over
  the ranks that registered (parallel/world.shrink) and carry on; rank 0 then issues a clean job
  so the nonce space is re-partitioned over the new ranks.
Resume: the leader persists {tip, extranonce} (miner_state.json); a restart on the same tip
continues the extranonce sequence, so no template searched before the restart is searched again.
"""
from __future__ import annotations

import datetime
import json
import os
import struct
import sys
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field

import numpy as np

from .. import core
from ..utils import log
from .search import (ALGO_EQUIHASH, ALGO_KAWPOW, ALGO_NAMES, ALGO_X16R, ALGO_X16RV2, EPOCH_PREBUILD_WINDOW,
                     FLAG_CLEAN, FLAG_IDLE, FLAG_STOP, WORK_SIZE, DeviceFault, DeviceHung, EquihashShare,
                     LegacyShare, SearchPipeline, SlotResult, Work, as_rank_device)

_core = core()

EXIT_DEVICE_HUNG = 75
EXIT_DEVICE_FAILED = 76
MAX_SHARES = {ALGO_KAWPOW: 16, ALGO_EQUIHASH: 4, ALGO_X16R: 16, ALGO_X16RV2: 16}
MAX_SHARES_PER_STEP = MAX_SHARES[ALGO_KAWPOW]
# job, work done, nshares, algo, device_us, aborted workgroups, collective wait us (previous step),
# consecutive failures, first resident epoch, resident epochs, status bits, device index
_REC_HEAD = struct.Struct("<QQIIIIIIIIIi")
_SHARE = {ALGO_KAWPOW: struct.Struct("<Q32s32s"),        # nonce, mix, final
          ALGO_EQUIHASH: struct.Struct("<Q1344s32s"),    # nonce, packed solution, block hash
          ALGO_X16R: struct.Struct("<Q32s"),             # nNonce, block hash
          ALGO_X16RV2: struct.Struct("<Q32s")}
RECORD_PAYLOAD = max(MAX_SHARES[a] * s.size for a, s in _SHARE.items())  # 5536
RECORD_SIZE = _REC_HEAD.size + RECORD_PAYLOAD                           # 5592
STATUS_RESULT, STATUS_ALIVE, STATUS_VOTE = 1, 2, 4  # VOTE: next-epoch light cache ready


class CollectiveError(RuntimeError):
    """A collective of the mining loop failed or timed out (a peer rank is gone or hung)."""


class DeviceEvicted(RuntimeError):
    """This rank's device failed `max_failures` windows in a row."""


@dataclass
class RankRecord:
    """One rank's gathered step record."""
    job_id: int = 0
    hashes: int = 0
    shares: list = field(default_factory=list)
    algo: int = ALGO_KAWPOW
    device_ms: float = 0.0
    aborted: int = 0
    coll_ms: float = 0.0
    failures: int = 0
    epochs: list = field(default_factory=list)
    has_result: bool = False
    alive: bool = True
    device: int = -1


def _as_record(r) -> RankRecord:
    if isinstance(r, RankRecord):
        return r
    job, hashes, shares = r  # (job_id, hashes, shares) tuples: tests, remote leader
    return RankRecord(job, hashes, list(shares), has_result=True)


def pack_record(res: SlotResult | None, *, coll_ms: float = 0.0, failures: int = 0, epochs=(),
                alive: bool = True, device: int = -1, vote: bool = False) -> bytes:
    out = bytearray(RECORD_SIZE)
    ep = sorted(epochs)
    lo, n = (ep[0], ep[-1] - ep[0] + 1) if ep else (0, 0)
    status = (STATUS_RESULT if res is not None else 0) | (STATUS_ALIVE if alive else 0) | (STATUS_VOTE if vote else 0)
    if res is None:
        _REC_HEAD.pack_into(out, 0, 0, 0, 0, 0, 0, 0, int(coll_ms * 1e3), failures, lo, n, status, device)
        return bytes(out)
    fmt = _SHARE[res.algo]
    shares = res.shares[:MAX_SHARES[res.algo]]
    _REC_HEAD.pack_into(out, 0, res.job_id, res.hashes, len(shares), res.algo, min(int(res.device_ms * 1e3), 2**32 - 1),
                        res.aborted, min(int(coll_ms * 1e3), 2**32 - 1), failures, lo, n, status, device)
    for i, s in enumerate(shares):
        off = _REC_HEAD.size + i * fmt.size
        if res.algo == ALGO_KAWPOW:
            fmt.pack_into(out, off, s.nonce, s.mix_hash, s.final_hash)
        elif res.algo == ALGO_EQUIHASH:
            fmt.pack_into(out, off, s.nonce, s.solution, s.block_hash)
        else:
            fmt.pack_into(out, off, s.nonce, s.block_hash)
    return bytes(out)


def record_totals(gathered: list[bytes]) -> tuple[int, int]:
    """(hashes, next-epoch votes) summed over the gathered records: the loop's counters ride in
    the record all-gather instead of an all-reduce of their own (one collective less per step)."""
    hashes = votes = 0
    for raw in gathered:
        _job, h, *_rest, status, _dev = _REC_HEAD.unpack_from(raw, 0)
        hashes += h
        votes += bool(status & STATUS_VOTE)
    return hashes, votes


def unpack_record(raw: bytes) -> RankRecord:
    from ..ops.kawpow import Share

    job, hashes, n, algo, dev_us, aborted, coll_us, failures, lo, nep, status, device = _REC_HEAD.unpack_from(raw, 0)
    fmt = _SHARE.get(algo, _SHARE[ALGO_KAWPOW])
    shares = []
    for i in range(min(n, MAX_SHARES.get(algo, 0))):
        vals = fmt.unpack_from(raw, _REC_HEAD.size + i * fmt.size)
        if algo == ALGO_KAWPOW:
            shares.append(Share(*vals))
        elif algo == ALGO_EQUIHASH:
            shares.append(EquihashShare(*vals))
        else:
            shares.append(LegacyShare(*vals))
    return RankRecord(job, hashes, shares, algo, dev_us / 1e3, aborted, coll_us / 1e3, failures,
                      list(range(lo, lo + nep)), bool(status & STATUS_RESULT), bool(status & STATUS_ALIVE), device)


class Comm:
    """The loop's collectives on the current world group, each bounded by a timeout.

    RCCL: tensors live on the GPU and the collectives are issued from a stream of their own, so
    they never queue behind the search kernel that is running on the search stream. gloo: host
    tensors. Without a process group (a single CPU rank) there is nothing to exchange. A world
    initialised with forced collectives (parallel/world.init(force_collectives=True)) runs them
    even at world size 1, so a one-GPU box executes the same RCCL path as an 8-GPU node."""

    def __init__(self, timeout_s: float):
        from ..parallel import world as W

        self.W = W
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.fail_at_step = int(os.environ.get("NODEXA_MINER_FAIL_COLLECTIVE_AT", "0"))  # test hook
        self.calls = 0
        self.rebind()

    def rebind(self) -> None:
        """Bind to the current world. The loop gets a communicator of its own (not the default
        group), so a failed one can be aborted (RCCL) and replaced without touching the default
        group or its rendezvous store."""
        self.w = self.W.get()
        self.active = self.w.collective
        self.gpu = self.w.backend == "nccl"
        self.stream = None
        self._buf: dict[str, tuple] = {}
        self.group = self.w.group
        if self.active:
            import torch

            self.torch = torch
            dist = self.W.dist
            if self.gpu:
                # the highest priority: its copies must not share a hardware queue with the search
                # stream, where they would wait behind the window queued for the next step and
                # drain the two-window pipeline every step (profiles/README r4b)
                self.stream = torch.cuda.Stream(device=self.w.device, priority=-16)
            if self.W.is_init_group(self.group):
                # gloo connects the group's full mesh under the group timeout, and ranks reach this
                # point seconds apart on a loaded host (a DAG build, a cold import): connect under the
                # rendezvous timeout. Every collective stays bounded by self.timeout (_wait), and a
                # dead gloo peer fails its pair at once.
                conn = self.timeout if self.gpu else max(self.timeout,
                                                         datetime.timedelta(seconds=self.W.rendezvous_timeout()))
                self.group = dist.new_group(ranks=list(range(self.w.world_size)), timeout=conn)

    def abort(self) -> None:
        """Tear down the loop's communicator after a failure: RCCL kernels still waiting for a dead
        peer are cancelled (ncclCommAbort); gloo needs nothing (its ops already raised)."""
        if self.gpu and self.group is not None:
            try:
                self.W.dist.distributed_c10d._abort_process_group(self.group)
            except Exception as e:  # noqa: BLE001 — best effort; the survivors re-form regardless
                log.log_printf(f"miner: aborting the failed communicator: {e}")
        if self.w.group is None:
            self.group = None  # rebind() makes a fresh loop communicator

    def _wait(self, work, what: str) -> None:
        try:
            ok = work.wait(timeout=self.timeout)
        except Exception as e:  # noqa: BLE001 — gloo raises on a closed peer, RCCL on timeout
            raise CollectiveError(f"{what}: {e}") from e
        if ok is False:
            raise CollectiveError(f"{what}: timed out")

    def _run(self, fn, what: str):
        self.calls += 1
        if self.fail_at_step and self.calls == self.fail_at_step:
            raise CollectiveError(f"{what}: timed out (injected, NODEXA_MINER_FAIL_COLLECTIVE_AT)")
        torch = self.torch
        if self.gpu:
            with torch.cuda.device(self.w.device), torch.cuda.stream(self.stream):
                out = fn()
                self.stream.synchronize()
                return out
        return fn()

    def _bufs(self, key: str, n: int):
        """Persistent (pinned host, device) byte buffers of a collective (RCCL): no allocation and
        no pageable copy per step."""
        b = self._buf.get(key)
        if b is None or b[0].numel() < n:
            torch = self.torch
            b = (torch.empty(n, dtype=torch.uint8).pin_memory(), torch.empty(n, dtype=torch.uint8, device=self.w.device))
            self._buf[key] = b
        return b[0][:n], b[1][:n]

    def broadcast(self, payload: bytes | None, size: int) -> bytes:
        if not self.active:
            return payload
        torch, dist = self.torch, self.W.dist

        def go():
            if self.gpu:
                host, dev = self._bufs("bcast", size)
                if self.w.rank == 0:
                    host.numpy()[:] = np.frombuffer(payload, dtype=np.uint8, count=size)
                    dev.copy_(host, non_blocking=True)
                self._wait(dist.broadcast(dev, src=self.w.global_rank(0), group=self.group, async_op=True), "broadcast")
                host.copy_(dev, non_blocking=True)
                self.stream.synchronize()
                return host.numpy().tobytes()
            t = torch.zeros(size, dtype=torch.uint8)
            if self.w.rank == 0:
                t.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
            self._wait(dist.broadcast(t, src=self.w.global_rank(0), group=self.group, async_op=True), "broadcast")
            return bytes(t.numpy().tobytes())

        return self._run(go, "broadcast")

    def all_gather(self, record: bytes) -> list[bytes]:
        if not self.active:
            return [record]
        torch, dist = self.torch, self.W.dist
        n, ws = len(record), self.w.world_size

        def go():
            if self.gpu:
                host, mine = self._bufs("rec", n)
                hout, out = self._bufs("gather", ws * n)
                host.numpy()[:] = np.frombuffer(record, dtype=np.uint8)
                mine.copy_(host, non_blocking=True)
                self._wait(dist.all_gather_into_tensor(out, mine, group=self.group, async_op=True), "all_gather")
                hout.copy_(out, non_blocking=True)
                self.stream.synchronize()
                raw = hout.numpy().tobytes()
            else:
                out = torch.empty(ws * n, dtype=torch.uint8)
                parts = list(out.view(ws, n).unbind(0))
                mine = torch.frombuffer(bytearray(record), dtype=torch.uint8)
                self._wait(dist.all_gather(parts, mine, group=self.group, async_op=True), "all_gather")
                raw = bytes(out.numpy().tobytes())
            return [raw[i * n:(i + 1) * n] for i in range(ws)]

        return self._run(go, "all_gather")

    def all_reduce_sum(self, vals: list[int]) -> list[int]:
        if not self.active:
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
    """Work per second over a sliding window (getmininginfo.hashespersec)."""

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
    until stopped) or `max_tries` units of work (hashes; Equihash: solutions) are spent."""
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
    header: bytes         # the work packet's header field
    boundary: bytes
    prev: bytes
    tx_updated: int
    created: float
    script: bytes
    algo: int = ALGO_KAWPOW
    tries: int = 0


def algo_for_time(params, t: int) -> int:
    """Which proof of work a header with nTime `t` carries (src/primitives/block.cpp:38-74 +
    the Equihash extension's activation)."""
    if t >= params.equihash_activation_time:
        return ALGO_EQUIHASH
    if t >= params.kawpow_activation_time:
        return ALGO_KAWPOW
    return ALGO_X16RV2 if t >= params.x16rv2_activation_time else ALGO_X16R


class ChainLeader:
    """Rank 0's side of the loop: templates -> work packets, shares -> blocks.

    Templates come from BlockAssembler (src/miner.cpp:123-256) with IncrementExtraNonce
    (:508-525) per job; a job is replaced when the tip moves, when the pool changed and the job is
    older than `refresh_s` (the reference's 60 s mempool check, src/miner.cpp:700-705), when a
    legacy job has spent its 2^28 nNonce values per rank, or when the world was re-partitioned.
    Every share is checked again before its block is built; only shares of a job whose parent is
    still the tip are submitted (the reference's "generated block is stale" check,
    ProcessBlockFound)."""

    def __init__(self, state, *, refresh_s: float = 10.0, target_bits: int = 0, on_block=None,
                 state_path: str | None = None):
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
        self.per_rank: dict[int, dict] = {}
        self.state_path = state_path
        self._resume = self._load_state()

    # ---------------------------------------------------------------- resume state
    def _load_state(self) -> dict:
        if not self.state_path or not os.path.exists(self.state_path):
            return {}
        try:
            with open(self.state_path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}

    def save_state(self) -> None:
        if not self.state_path:
            return
        data = {"tip": _core.u256_hex(self.extranonce.prev) if self.extranonce.prev else None,
                "extranonce": self.extranonce.n, "job": self.job_seq, "time": int(time.time())}
        tmp = self.state_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, self.state_path)

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

    def fail(self, why: str) -> None:
        """The loop cannot mine any more (every device evicted): end the request with an error."""
        with self.lock:
            req = self.request
        if req is not None and not req.done.is_set():
            req.error = why
            req.done.set()

    def shutdown(self) -> None:
        self.stop_mining()
        self.stopping = True

    # ---------------------------------------------------------------- called from the loop thread
    def _new_job(self, req: MiningRequest) -> Job:
        from ..chain.header import to_progpow
        from .assembler import BlockAssembler

        st = self.state
        tpl = BlockAssembler(st).create_new_block(req.script)
        blk = tpl.block
        hdr = blk.header
        if self.extranonce.prev != hdr.prev and self._resume.get("tip") == _core.u256_hex(hdr.prev):
            # a restart on the tip of a saved run: continue its extranonce sequence
            self.extranonce.prev, self.extranonce.n = hdr.prev, int(self._resume.get("extranonce", 0))
        self.extranonce.increment(blk, tpl.height)
        hdr = blk.header
        algo = algo_for_time(st.params, hdr.time)
        target = tpl.target if self.miner_target is None else min(tpl.target, self.miner_target)
        if algo == ALGO_KAWPOW:
            header = to_progpow(hdr.kawpow_header_hash())
        elif algo == ALGO_EQUIHASH:
            header = hdr.kawpow_input()  # version (with the extension bit), prev, merkle, time, bits, height
        else:
            header = hdr.legacy80()
        self.job_seq += 1
        job = Job(self.job_seq, blk, tpl.height, header, target.to_bytes(32, "big"), hdr.prev,
                  st.transactions_updated, time.time(), req.script, algo)
        self.jobs[job.job_id] = job
        while len(self.jobs) > 8:
            self.jobs.popitem(last=False)
        try:
            self.save_state()
        except OSError:
            pass
        return job

    def next_work(self, repartitioned: bool = False) -> Work:
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
                 or (st.transactions_updated != cur.tx_updated and time.time() - cur.created > self.refresh_s)
                 or (cur.algo in (ALGO_X16R, ALGO_X16RV2) and cur.tries >= 1 << 28))
        if not stale:
            return Work(cur.header, cur.boundary, cur.height, cur.job_id, 0, 0, cur.algo)
        job = self._new_job(req)
        return Work(job.header, job.boundary, job.height, job.job_id, 0, FLAG_CLEAN, job.algo)

    def _rank_stats(self, r: int) -> dict:
        return self.per_rank.setdefault(r, {"shares": 0, "stale_shares": 0, "bad_shares": 0, "blocks": 0})

    def _check_share(self, job: Job, sh) -> bool:
        if job.algo == ALGO_KAWPOW:
            return sh.verify_full(job.height, job.header[:32], job.boundary)
        if job.algo == ALGO_EQUIHASH:
            from .search import equihash_block_hash

            p = _core.EquihashParams(200, 9)
            inp = job.header + sh.nonce256()
            ok = bool(_core.equihash_verify(p, inp, _core.equihash_unpack(p, sh.solution))[0])
            bh = equihash_block_hash(job.header, sh.nonce, sh.solution)
            return ok and bh == sh.block_hash and int.from_bytes(bh, "little") <= int.from_bytes(job.boundary, "big")
        return int.from_bytes(sh.block_hash, "little") <= int.from_bytes(job.boundary, "big")

    def _block_for(self, job: Job, sh):
        from ..chain.header import from_progpow

        act = self.state.params.kawpow_activation_time
        blk = _core.Block.deserialize(job.block.serialize(act), act)
        hdr = blk.header
        if job.algo == ALGO_KAWPOW:
            hdr.nonce64 = sh.nonce
            hdr.mix_hash = from_progpow(sh.mix_hash)
        elif job.algo == ALGO_EQUIHASH:
            hdr.nonce256 = sh.nonce256()
            hdr.solution = sh.solution
        else:
            hdr.nonce = sh.nonce
        blk.header = hdr
        return blk

    def on_results(self, records) -> None:
        records = [_as_record(r) for r in records]
        req = self.request
        for r, rec in enumerate(records):
            job = self.jobs.get(rec.job_id)
            if job is not None:
                job.tries += rec.hashes
        if req is None:
            return
        req.tries += sum(rec.hashes for rec in records)
        st = self.state
        for r, rec in enumerate(records):
            rs = self._rank_stats(r)
            for sh in rec.shares:
                if req.done.is_set():
                    break
                self.stats["shares"] += 1
                rs["shares"] += 1
                job = self.jobs.get(rec.job_id)
                if job is None or job.prev != st.tip().hash:
                    self.stats["stale_shares"] += 1
                    rs["stale_shares"] += 1
                    continue
                if not self._check_share(job, sh):
                    self.stats["bad_shares"] += 1
                    rs["bad_shares"] += 1
                    log.log_printf(f"miner: {ALGO_NAMES[job.algo]} share nonce {sh.nonce:#x} of job {rec.job_id} "
                                   f"(rank {r}) failed the host check; dropped")
                    continue
                blk = self._block_for(job, sh)
                res = st.process_new_block(blk)
                if not res.ok:
                    self.stats["rejected"] += 1
                    log.log_printf(f"miner: block of job {rec.job_id} rejected: {res.reject}")
                    if req.blocks is not None:  # generateBlocks: "ProcessNewBlock, block not accepted"
                        req.error = f"ProcessNewBlock, block not accepted: {res.reject}"
                        req.done.set()
                        break
                    continue
                bh = st.block_hash(blk.header)
                self.stats["blocks"] += 1
                rs["blocks"] += 1
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
    """A fixed synthetic job (bench.py): the same loop, no chain. Shares are kept for the host
    re-check after the timed region."""

    def __init__(self, work: Work, keep: int = 64):
        self.work = Work(work.header, work.boundary, work.height, work.job_id or 1, work.nonce_base, 0, work.algo)
        self.first = True
        self.keep = keep
        self.shares: list = []
        self.records = 0
        self.stopping = False

    def next_work(self, repartitioned: bool = False) -> Work:
        if self.stopping:
            return Work(flags=FLAG_STOP)
        if self.first or repartitioned:
            self.first = False
            w = self.work
            return Work(w.header, w.boundary, w.height, w.job_id, w.nonce_base, FLAG_CLEAN, w.algo)
        return self.work

    def on_results(self, records) -> None:
        for rec in (_as_record(r) for r in records):
            self.records += rec.has_result
            if len(self.shares) < self.keep:
                self.shares.extend(rec.shares[:self.keep - len(self.shares)])

    def shutdown(self) -> None:
        self.stopping = True


class MiningService:
    """The per-rank mining loop (see the module docstring). Rank 0 passes a leader."""

    def __init__(self, device, leader=None, *, window: int = 1 << 25, watchdog_s: float = 120.0,
                 collective_timeout_s: float = 60.0, grace_s: float | None = None, idle_sleep_s: float = 0.02,
                 record_windows: bool = False, max_failures: int = 3):
        from ..parallel import world as W

        self.W = W
        self.dev = as_rank_device(device)
        self.leader = leader
        self.window = int(window)
        self.pipe = SearchPipeline(self.dev, watchdog_s)
        self.comm = Comm(collective_timeout_s)
        self.collective_timeout_s = float(collective_timeout_s)
        self.grace_s = float(grace_s) if grace_s is not None else 2 * self.collective_timeout_s + 1
        self.idle_sleep_s = float(idle_sleep_s)
        self.max_failures = int(max_failures)
        self.work = Work()
        self.cursor = 0
        self.rate = RateMeter()
        self.hashes_total = 0
        self.rank_hashes: dict[int, int] = {}
        self.rank_info_raw: dict[int, dict] = {}
        self.rank_rates: dict[int, RateMeter] = {}
        self.steps = 0
        self.membership = 0
        self.repartitioned = False
        self.windows: list[tuple[int, int, int]] | None = [] if record_windows else None
        self._light_thread: threading.Thread | None = None
        self._thread: threading.Thread | None = None
        self.error: BaseException | None = None
        self.last_step_ms = 0.0
        self.coll_ms = 0.0
        self.last_end_ms = 0.0  # device clock of the last window this rank took (SlotResult.end_ms)
        self.failures = 0          # consecutive failed windows on this rank
        self.total_failures = 0
        self.dev_alive = True
        self.last_error = ""

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
        if w.idle or w.algo != ALGO_KAWPOW or w.height % _core.EPOCH_LENGTH < _core.EPOCH_LENGTH - EPOCH_PREBUILD_WINDOW:
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

    def _window_start(self, w: Work) -> int:
        if w.algo in (ALGO_X16R, ALGO_X16RV2):
            return ((self.rank & 0xF) << 28) | (self.cursor & 0x0FFFFFFF)
        return (w.nonce_base + (self.rank << 56) + self.cursor) & 0xFFFFFFFFFFFFFFFF

    def _device_failure(self, err: Exception) -> None:
        self.failures += 1
        self.total_failures += 1
        self.last_error = f"{type(err).__name__}: {err}"
        log.log_printf(f"miner rank {self.rank}: window failed ({self.last_error}), {self.failures} in a row")
        if self.failures >= self.max_failures and self.dev_alive:
            self.dev_alive = False
            log.log_printf(f"miner rank {self.rank}: device evicted after {self.failures} failed windows")
            try:
                self.pipe.drain()
            except Exception:  # noqa: BLE001 — the device is being given up
                self.pipe.inflight = None
            if self.leader is None:
                raise DeviceEvicted(self.last_error)

    def step(self) -> bool:
        """One iteration of the loop on this rank; False once a stop packet has been processed."""
        t0 = time.perf_counter()
        w = self.work
        res = None
        try:
            if w.idle or not self.dev_alive:
                res = self.pipe.drain() if self.pipe.inflight is not None else None
                if res is None:
                    time.sleep(self.idle_sleep_s)
            else:
                count = self.dev.window_for(w, self.window)
                start = self._window_start(w)
                if self.windows is not None:
                    self.windows.append((w.job_id, start, count))
                self.cursor += count  # before the step: a window that fails was still searched once
                res = self.pipe.step(w, start, count)
            if res is not None:
                self.failures = 0
                self.last_end_ms = res.end_ms
        except DeviceFault as e:
            self._device_failure(e)
            res = None
        vote = self._next_epoch_vote()
        rec = pack_record(res, coll_ms=self.coll_ms, failures=self.failures, epochs=self.dev.resident_epochs(),
                          alive=self.dev_alive, device=int(getattr(self.dev, "device", -1)), vote=bool(vote))
        tc = time.perf_counter()
        gathered = self.comm.all_gather(rec)
        coll = time.perf_counter() - tc
        hashes, votes = record_totals(gathered)
        self.hashes_total += hashes
        self.rate.add(hashes)
        if vote and votes == self.world_size:
            # every rank holds the light cache: all start the (collective) build on this step
            self.dev.prebuild(w.epoch + 1)
            self._light_thread = None
        payload = None
        if self.leader is not None:
            records = [unpack_record(r) for r in gathered]
            now = time.monotonic()
            for i, rec_i in enumerate(records):
                self.rank_hashes[i] = self.rank_hashes.get(i, 0) + rec_i.hashes
                self.rank_rates.setdefault(i, RateMeter()).add(rec_i.hashes, now)
                info = self.rank_info_raw.setdefault(i, {"aborted": 0, "windows": 0})
                info.update(alive=rec_i.alive, failures=rec_i.failures, epochs=rec_i.epochs, device=rec_i.device,
                            coll_ms=rec_i.coll_ms)
                if rec_i.has_result:
                    info["windows"] += 1
                    info["aborted"] += rec_i.aborted
                    info.update(algo=rec_i.algo, device_ms=rec_i.device_ms)
            self.leader.on_results(records)
            if self.world_size == 1 and not self.dev_alive and hasattr(self.leader, "fail"):
                self.leader.fail("no mining device left (all evicted): " + self.last_error)
            payload = self.leader.next_work(self.repartitioned).pack()
            self.repartitioned = False
        tc = time.perf_counter()
        new = Work.unpack(self.comm.broadcast(payload, WORK_SIZE))
        self.coll_ms = (coll + time.perf_counter() - tc) * 1e3
        if new.job_id != w.job_id:
            self.cursor = 0
        if new.flags & FLAG_CLEAN or new.idle:
            self.dev.abort()  # the window queued for the old job stops on the device
        self.work = new
        self.steps += 1
        self.last_step_ms = (time.perf_counter() - t0) * 1e3
        return not new.stop

    # ---------------------------------------------------------------- observability
    def rank_info(self) -> list[dict]:
        """getmininginfo.gpus[]: one entry per rank of the world (rank 0 only)."""
        out = []
        stats = getattr(self.leader, "per_rank", {}) if self.leader is not None else {}
        for r in range(self.world_size):
            info = self.rank_info_raw.get(r, {})
            rs = stats.get(r, {})
            algo = info.get("algo", self.work.algo)
            shares, stale = rs.get("shares", 0), rs.get("stale_shares", 0)
            rate = self.rank_rates[r].rate() if r in self.rank_rates else 0.0
            out.append({
                "rank": r,
                "device": info.get("device", -1),
                "alive": info.get("alive", True) if r else self.dev_alive,
                "algo": ALGO_NAMES[algo] if algo < len(ALGO_NAMES) else str(algo),
                ("solutionspersec" if algo == ALGO_EQUIHASH else "hashespersec"): round(rate, 1),
                "mhs": round(rate / 1e6, 3) if algo != ALGO_EQUIHASH else None,
                "hashes": int(self.rank_hashes.get(r, 0)),
                "shares": shares,
                "stale_shares": stale,
                "stale_rate": round(stale / shares, 4) if shares else 0.0,
                "bad_shares": rs.get("bad_shares", 0),
                "blocks": rs.get("blocks", 0),
                "epochs_resident": info.get("epochs", []),
                "last_device_ms": round(info.get("device_ms", 0.0), 3),
                "last_step_ms": round(self.last_step_ms, 3),
                "collective_ms": round(info.get("coll_ms", 0.0), 3),
                "aborted_workgroups": info.get("aborted", 0),
                "windows": info.get("windows", 0),
                "failures": info.get("failures", 0),
            })
        return out

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


class Miner:
    """The node's miner front-end (node.miner): generate / generatetoaddress / setgenerate /
    getmininginfo on top of the mining service's leader. Every proof of work and every device
    goes through the one loop; there is no second, thread-per-backend miner."""

    def __init__(self, state, service: MiningService):
        from ..utils.metrics import REGISTRY

        self.state = state
        self.service = service
        self.leader: ChainLeader = service.leader
        self.metrics = REGISTRY
        self._req: MiningRequest | None = None
        self.generating = False
        self._last_hashes = 0
        self._last_shares = 0

    @classmethod
    def local(cls, state, *, window: int = 4096, fail_rate: float = 0.0, drop_rate: float = 0.0,
              max_failures: int = 3, watchdog_s: float = 120.0, state_path: str | None = None,
              target_bits: int = 0, start: bool = True) -> "Miner":
        """A single-rank miner on this host's CPU devices (CPU-only nodes, tests)."""
        from .search import CpuSearchDevice, FaultInjectingDevice, RankDevice

        dev = RankDevice(CpuSearchDevice(max_window=window))
        if fail_rate or drop_rate:
            dev = FaultInjectingDevice(dev, fail_rate, drop_rate, seed=0)
        leader = ChainLeader(state, state_path=state_path, target_bits=target_bits)
        svc = MiningService(dev, leader, window=window, watchdog_s=watchdog_s, max_failures=max_failures)
        return cls(state, svc.start() if start else svc)

    @property
    def hashrate(self) -> float:
        """getmininginfo.hashespersec: the rate summed over every rank's gathered record
        (src/miner.cpp:685-687)."""
        return self.service.hashrate()

    def workers(self) -> list[dict]:
        return [{"worker": g["rank"], "backend": f"{getattr(self.service.dev, 'name', 'dev')}-rank{g['rank']}",
                 "alive": g["alive"], "hashes": g["hashes"], "blocks": g["blocks"], "failures": g["failures"]}
                for g in self.service.rank_info()]

    def _export_metrics(self) -> None:
        h, s = self.service.hashes_total, self.leader.stats["shares"]
        if h > self._last_hashes:
            self.metrics.inc("miner_hashes_total", h - self._last_hashes, worker="service")
        if s > self._last_shares:
            self.metrics.inc("miner_shares_total", s - self._last_shares, worker="service")
        self._last_hashes, self._last_shares = h, s

    def generate(self, script_pubkey: bytes, nblocks: int, max_tries: int = 1_000_000) -> list[str]:
        """generateBlocks: the new block hashes (display hex), mined by the service."""
        svc = self.service
        if svc.error is not None:
            raise RuntimeError(f"miner service stopped: {svc.error}")
        req = self.leader.mine(script_pubkey, blocks=nblocks, max_tries=max_tries)
        while not req.done.wait(0.2):
            if svc.error is not None:
                raise RuntimeError(f"miner service stopped: {svc.error}")
        self._export_metrics()
        for _ in req.found:
            self.metrics.inc("miner_blocks_total", 1, worker="service")
        if req.error is not None and not req.found:
            if req.error == "superseded":
                return []
            raise RuntimeError(req.error)
        return list(req.found)

    def set_generate(self, on: bool, script_pubkey: bytes | None = None) -> None:
        self.stop()
        if not on:
            return
        if script_pubkey is None:
            raise ValueError("setgenerate true needs -miningaddress")
        self._req = self.leader.mine(script_pubkey)  # until setgenerate false
        self.generating = True

    def stop(self) -> None:
        if self._req is not None:
            self.leader.stop_mining()
            for _ in self._req.found:
                self.metrics.inc("miner_blocks_total", 1, worker="service")
            self._req = None
        self._export_metrics()
        self.generating = False

    def close(self) -> None:
        """Node shutdown: stop mining and end the service loop (its stop packet ends every rank)."""
        self.stop()
        self.service.stop()


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


def make_rank_device(cpu: bool, device_index: int | None = None, collective_dag: bool = False, window: int = 4096,
                     fail_rate: float = 0.0, drop_rate: float = 0.0, seed: int = 0, eq_window: int = 1):
    """This rank's RankDevice: GPU KawPow + GPU Equihash (built on first use) + GPU X16R, or the
    host equivalents; -gpufailrate / -dropshare wrap it."""
    from .equihash_search import EquihashCpuDevice
    from .search import CpuSearchDevice, FaultInjectingDevice, RankDevice

    if cpu:
        dev = RankDevice(CpuSearchDevice(max_window=window), EquihashCpuDevice(eq_window))
    else:
        from .equihash_search import EquihashGpuDevice
        from .search import GpuSearchDevice, LegacyGpuDevice

        idx = int(device_index or 0)
        dev = RankDevice(GpuSearchDevice(idx, collective_dag=collective_dag),
                         equihash_factory=lambda: EquihashGpuDevice(idx), legacy=LegacyGpuDevice(idx))
    if fail_rate or drop_rate:
        dev = FaultInjectingDevice(dev, fail_rate, drop_rate, seed=seed)
    return dev


def follower_main() -> int:
    """Entry point of ranks >= 1 (spawned by the node or launched by torchrun)."""
    from ..parallel import world as W

    cpu = os.environ.get("NODEXA_MINER_CPU", "0") == "1"
    dev_index = os.environ.get("NODEXA_MINER_DEVICE")
    timeout = float(os.environ.get("NODEXA_MINER_COLLECTIVE_TIMEOUT", "60"))
    watchdog = float(os.environ.get("NODEXA_MINER_WATCHDOG", "120"))
    window = int(os.environ.get("NODEXA_MINER_WINDOW", str(1 << 25)))
    W.init(use_gpu=not cpu, device_index=None if dev_index is None else int(dev_index),
           timeout_s=max(int(timeout), W.rendezvous_timeout()), elastic=True, collective_timeout_s=timeout)
    w = W.get()
    dev = make_rank_device(cpu, w.device.index if not cpu else None, collective_dag=w.collective, window=window,
                           fail_rate=float(os.environ.get("NODEXA_MINER_FAILRATE", "0") or 0),
                           drop_rate=float(os.environ.get("NODEXA_MINER_DROPSHARE", "0") or 0), seed=w.rank)
    hang = int(os.environ.get("NODEXA_MINER_HANG_AFTER", "0"))
    if hang > 0:  # fault injection for the failure-handling tests
        from .search import HangingDevice

        dev = HangingDevice(dev, hang)
    wlog = os.environ.get("NODEXA_MINER_WINDOWS_LOG")
    svc = MiningService(dev, None, window=window, watchdog_s=watchdog, collective_timeout_s=timeout,
                        record_windows=bool(wlog), max_failures=int(os.environ.get("NODEXA_MINER_MAXFAILURES", "3")))

    def dump():
        if wlog:
            with open(wlog, "w") as f:
                json.dump({"rank": svc.rank, "world_size": svc.world_size, "windows": svc.windows,
                           "steps": svc.steps, "hashes_total": svc.hashes_total,
                           "failures": svc.total_failures}, f)

    try:
        svc.run()
    except DeviceHung as e:
        log.log_printf(f"miner rank {W.get().rank}: {e}; exiting so the survivors re-partition")
        dump()
        os._exit(EXIT_DEVICE_HUNG)
    except DeviceEvicted as e:
        log.log_printf(f"miner rank {W.get().rank}: device evicted ({e}); exiting so the survivors re-partition")
        dump()
        os._exit(EXIT_DEVICE_FAILED)
    except RuntimeError as e:
        log.log_printf(f"miner rank {W.get().rank}: {e}")
        dump()
        return 3
    dump()
    W.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(follower_main())
