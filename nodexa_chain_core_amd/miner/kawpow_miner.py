"""KawPow mining: PoW backends and the miner controller.

Parity: generateBlocks (src/rpc/mining.cpp:117-173: template -> extranonce ->
nonce loop with CheckProofOfWork(GetHashFull) -> ProcessNewBlock),
GenerateClores / CloreMiner (src/miner.cpp:566-759: background miner threads,
nHashesPerSec for getmininginfo). Fixed here: the reference's internal miner
bumps the 32-bit nNonce, which KawPow headers do not serialize or hash
(SURVEY §3.6); this controller always searches nNonce64.

Two ways to mine:
  * the mining service (miner/service.py) — the MI355X path and the only KawPow path of a GPU
    node: one process per GPU in one torch.distributed world (RCCL), a pipelined 2^25-nonce
    search loop per GPU, rank 0 (this node) turning shares into blocks. `MinerController` then
    only forwards generate / setgenerate / getmininginfo to the service's leader.
  * host backends in threads — CpuKawpowBackend (the reference-equivalent light-mode search,
    progpow::search_light) for CPU-only nodes, and the host X16R / X16RV2 search for templates
    before the KawPow activation.
"""
from __future__ import annotations

import threading
import time

from .. import core
from ..chain.header import from_progpow, to_progpow
from ..chain.state import ChainState
from ..utils import log, sync
from .assembler import BlockAssembler, ExtraNonce

_core = core()


class CpuKawpowBackend:
    name = "cpu"

    def __init__(self, threads: int = 1):
        self.threads = max(1, int(threads))

    def search(self, block_number: int, header_hash: bytes, boundary: bytes, start: int, count: int):
        ctx = _core.get_epoch_context(block_number // _core.EPOCH_LENGTH)
        ok, nonce, fin, mix = _core.kawpow_search_light(ctx, block_number, header_hash, boundary, start, count)
        return (nonce, mix, fin) if ok else None


class InjectedFault(RuntimeError):
    """A simulated device failure raised by FaultInjector (-gpufailrate)."""


class FaultInjector:
    """Test-only fault injection around a PoW backend (SURVEY §5 `-gpufailrate` /
    `-dropshare`): each search raises InjectedFault with probability `fail_rate`, and a
    found share is silently dropped with probability `drop_rate` (the window then reads
    as "no share", like a share lost between device and host)."""

    def __init__(self, backend, fail_rate: float = 0.0, drop_rate: float = 0.0, seed: int | None = None):
        import random

        self.inner = backend
        self.fail_rate, self.drop_rate = float(fail_rate), float(drop_rate)
        self.rng = random.Random(seed)
        self.dropped = 0

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def search(self, *a, **kw):
        if self.fail_rate and self.rng.random() < self.fail_rate:
            raise InjectedFault(f"injected device fault on {getattr(self.inner, 'name', '?')}")
        res = self.inner.search(*a, **kw)
        if res is not None and self.drop_rate and self.rng.random() < self.drop_rate:
            self.dropped += 1
            return None
        return res


class WorkerHealth:
    """Per-backend state for the watchdog: heartbeats, consecutive failures, eviction."""

    def __init__(self, index: int, backend):
        self.index = index
        self.backend = backend
        self.label = f"{getattr(backend, 'name', 'be')}{getattr(backend, 'device', index)}"
        self.alive = True
        self.failures = 0          # consecutive
        self.total_failures = 0
        self.last_error = ""
        self.heartbeat = time.time()
        self.busy_since: float | None = None
        self.hashes = 0
        self.blocks = 0

    def as_dict(self) -> dict:
        return {"worker": self.index, "backend": self.label, "alive": self.alive, "failures": self.total_failures,
                "last_error": self.last_error, "hashes": self.hashes, "blocks": self.blocks}


class MinerController:
    """generate / generatetoaddress / setgenerate on top of one or more PoW backends.

    Background mining runs one host thread per backend (GPU) over disjoint nNonce64
    ranges: worker k of n alive workers starts at k << 56 (the same deterministic
    partition bench.py uses across ranks). Failure handling:
      * every search that raises counts a failure; `max_failures` consecutive ones, or
        a search that outlives `watchdog_s` (a hung kernel), evict the worker;
      * eviction re-partitions the nonce space over the surviving workers (their rank
        among the alive set changes at the next template) — the elastic analogue of
        rebuilding the communicator without the failed GPU;
      * shares are re-verified on the host by the backends before they are used.
    Resume: with a `state_path`, each worker's {tip, extranonce, nonce cursor} is saved
    periodically; a restart on the same tip continues the extranonce sequence, so no
    template (and no nonce range under it) searched before the restart is searched again."""

    def __init__(self, state: ChainState, backends: list, *, max_failures: int = 3, watchdog_s: float = 120.0,
                 state_path: str | None = None, service=None):
        from ..utils.metrics import REGISTRY

        self.state = state
        self.backends = backends
        self.service = service  # miner/service.MiningService with a ChainLeader (GPU nodes)
        self._service_req = None
        self.metrics = REGISTRY
        self.health = [WorkerHealth(i, b) for i, b in enumerate(backends)]
        self.max_failures, self.watchdog_s = int(max_failures), float(watchdog_s)
        self.state_path = state_path
        self.hashes_done = 0
        self._hashrate = 0.0
        self._rate_t0 = time.time()
        self._threads: list[threading.Thread] = []
        self._stop = threading.Event()
        self._lock = sync.make_lock("cs_miner")
        self._cursors: dict[int, dict] = self._load_state()
        self.generating = False

    # --------------------------------------------------------------- helpers
    @property
    def hashrate(self) -> float:
        """getmininginfo.hashespersec: the service's all-reduced rate over every rank, else the
        host threads' rate (src/miner.cpp:685-687)."""
        if self.service is not None and (self._service_req is not None or self._hashrate == 0.0):
            return self.service.hashrate()
        return self._hashrate

    def workers(self) -> list[dict]:
        if self.service is None:
            return [h.as_dict() for h in self.health]
        svc = self.service
        return [{"worker": r, "backend": f"{getattr(svc.dev, 'name', 'dev')}-rank{r}", "alive": True,
                 "hashes": int(svc.rank_hashes.get(r, 0)),
                 "blocks": svc.leader.stats["blocks"] if r == 0 and svc.leader is not None else 0}
                for r in range(svc.world_size)]

    def _kawpow_template_time(self) -> bool:
        tip = self.state.tip()
        return max(tip.median_time_past() + 1, int(time.time())) >= self.state.params.kawpow_activation_time

    def _service_generate(self, script_pubkey: bytes, nblocks: int, max_tries: int) -> list[str] | None:
        """generate through the mining service; None if the template is pre-KawPow (host search)."""
        svc = self.service
        if svc.error is not None:
            raise RuntimeError(f"miner service stopped: {svc.error}")
        req = svc.leader.mine(script_pubkey, blocks=nblocks, max_tries=max_tries)
        while not req.done.wait(0.5):
            if svc.error is not None:
                raise RuntimeError(f"miner service stopped: {svc.error}")
        if req.error is not None and "KawPow activation" in req.error:
            return None
        if req.error is not None and not req.found:
            raise RuntimeError(req.error)
        for h in req.found:
            self.metrics.inc("miner_blocks_total", 1, worker="service")
        return list(req.found)

    def _account(self, n: int, worker: int | None = None) -> None:
        with self._lock:
            self.hashes_done += n
            dt = time.time() - self._rate_t0
            if dt > 4.0:
                self._hashrate = self.hashes_done / dt
                self.hashes_done = 0
                self._rate_t0 = time.time()
        label = self.health[worker].label if worker is not None else "generate"
        if worker is not None:
            self.health[worker].hashes += n
        self.metrics.inc("miner_hashes_total", n, worker=label)

    def alive_workers(self) -> list[WorkerHealth]:
        return [h for h in self.health if h.alive]

    def nonce_base(self, worker: int) -> int:
        """Deterministic partition over the alive workers: rank r of n -> r << 56."""
        alive = [h.index for h in self.alive_workers()]
        rank = alive.index(worker) if worker in alive else worker
        return (rank & 0xFF) << 56

    def evict(self, worker: int, reason: str) -> None:
        h = self.health[worker]
        if not h.alive:
            return
        h.alive = False
        h.last_error = reason
        self.metrics.inc("miner_evictions_total", 1, worker=h.label)
        log.log_printf(f"miner: evicting worker {worker} ({h.label}): {reason}; "
                       f"{len(self.alive_workers())} worker(s) left, nonce space re-partitioned")

    def _load_state(self) -> dict[int, dict]:
        import json
        import os

        if not self.state_path or not os.path.exists(self.state_path):
            return {}
        try:
            with open(self.state_path) as f:
                return {int(k): v for k, v in json.load(f).get("workers", {}).items()}
        except (OSError, ValueError):
            return {}

    def save_state(self) -> None:
        import json
        import os

        if not self.state_path:
            return
        with self._lock:
            data = {"workers": {str(k): v for k, v in self._cursors.items()}, "time": int(time.time())}
        tmp = self.state_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, self.state_path)

    def resume_extranonce(self, worker: int, tip_hex: str) -> int:
        c = self._cursors.get(worker)
        return int(c.get("extranonce", 0)) if c and c.get("tip") == tip_hex else 0

    def _set_cursor(self, worker: int, tip_hex: str, extranonce: int, cursor: int) -> None:
        with self._lock:
            self._cursors[worker] = {"tip": tip_hex, "extranonce": int(extranonce), "cursor": int(cursor)}

    def mine_one(self, script_pubkey: bytes, backend, max_tries: int, extranonce: ExtraNonce,
                 nonce_start: int = 0, stop: threading.Event | None = None, worker: int | None = None):
        """Build a template and search nNonce64 in [nonce_start, +max_tries). Returns (block, tries)."""
        asm = BlockAssembler(self.state)
        tpl = asm.create_new_block(script_pubkey)
        blk = tpl.block
        xn = extranonce.increment(blk, tpl.height)
        hdr = blk.header
        if hdr.time < self.state.params.kawpow_activation_time:
            return self._mine_legacy(blk, tpl, max_tries, nonce_start, stop, worker)
        header_hash = to_progpow(hdr.kawpow_header_hash())
        boundary = tpl.target.to_bytes(32, "big")
        chunk = 1 << 16
        tried = 0
        tip_hex = _core.u256_hex(hdr.prev)
        while tried < max_tries and not (stop and stop.is_set()):
            n = min(chunk, max_tries - tried)
            h = self.health[worker] if worker is not None else None
            if h is not None:
                h.busy_since = time.time()
            res = backend.search(tpl.height, header_hash, boundary, nonce_start + tried, n)
            if h is not None:
                h.busy_since = None
                h.heartbeat = time.time()
                h.failures = 0
                self._set_cursor(worker, tip_hex, xn, nonce_start + tried + n)
            if res is None:
                tried += n
                self._account(n, worker)
                continue
            nonce, mix, fin = res
            self._account(nonce - (nonce_start + tried) + 1, worker)
            self.metrics.inc("miner_shares_total", 1, worker=h.label if h else "generate")
            hdr.nonce64 = nonce
            hdr.mix_hash = from_progpow(mix)
            blk.header = hdr
            return blk, tried + (nonce - nonce_start - tried) + 1
        return None, tried

    def _mine_legacy(self, blk, tpl, max_tries: int, nonce_start: int, stop, worker: int | None = None):
        """Pre-KawPow template (X16R / X16RV2 by nTime, src/primitives/block.cpp:38-55):
        the reference's generateBlocks bumps the 32-bit nNonce (src/rpc/mining.cpp:141-149).
        Native multi-threaded search (csrc/pow/x16r.cpp) in 64k-nonce windows."""
        hdr = blk.header
        v2 = hdr.time >= self.state.params.x16rv2_activation_time
        target = tpl.target.to_bytes(32, "little")
        tried = 0
        start = nonce_start & 0xFFFFFFFF
        while tried < max_tries and not (stop and stop.is_set()):
            n = min(1 << 16, max_tries - tried, (1 << 32) - start)
            hdr.nonce = 0
            res, hashes = _core.x16r_search(hdr.legacy80(), v2, target, start, n)
            self._account(hashes, worker)
            if res is not None:
                hdr.nonce = res[0]
                blk.header = hdr
                return blk, tried + (res[0] - start) + 1
            tried += n
            start += n
            if start >= 1 << 32:
                break
        return None, tried

    def generate(self, script_pubkey: bytes, nblocks: int, max_tries: int = 1_000_000) -> list[str]:
        """generateBlocks: returns the new block hashes (display hex). Uses the first alive
        backend; a backend that raises is evicted and the next one takes over."""
        if self.service is not None and self._kawpow_template_time():
            found = self._service_generate(script_pubkey, nblocks, max_tries)
            if found is not None:
                return found
        out: list[str] = []
        extranonce = ExtraNonce()
        while len(out) < nblocks and max_tries > 0:
            alive = self.alive_workers()
            if not alive:
                raise RuntimeError("no mining backend left (all evicted)")
            h = alive[0]
            try:
                blk, tried = self.mine_one(script_pubkey, h.backend, max_tries, extranonce, worker=h.index)
            except Exception as e:  # noqa: BLE001 — device faults surface as arbitrary errors
                self._failure(h.index, e)
                continue
            max_tries -= tried
            if blk is None:
                break
            st = self.state.process_new_block(blk)
            if not st.ok:
                raise RuntimeError(f"ProcessNewBlock, block not accepted: {st.reject}")
            bh = self.state.block_hash(blk.header)
            h.blocks += 1
            self.metrics.inc("miner_blocks_total", 1, worker=h.label)
            self.state._emit("block_found", bh)
            out.append(_core.u256_hex(bh))
        return out

    def _failure(self, worker: int, err: Exception) -> None:
        h = self.health[worker]
        h.failures += 1
        h.total_failures += 1
        h.last_error = f"{type(err).__name__}: {err}"
        h.busy_since = None
        self.metrics.inc("miner_failures_total", 1, worker=h.label)
        log.log_printf(f"miner worker {worker} ({h.label}) error #{h.failures}: {err}")
        if h.failures >= self.max_failures:
            self.evict(worker, f"{h.failures} consecutive failures, last: {h.last_error}")

    # --------------------------------------------------------------- background mining
    def set_generate(self, on: bool, script_pubkey: bytes | None = None) -> None:
        self.stop()
        if not on:
            return
        if script_pubkey is None:
            raise ValueError("setgenerate true needs -miningaddress")
        if self.service is not None and self._kawpow_template_time():
            self._service_req = self.service.leader.mine(script_pubkey)  # until setgenerate false
            self.generating = True
            return
        self._stop.clear()
        self.generating = True
        for h in self.alive_workers():
            t = threading.Thread(target=self._loop, args=(h.backend, script_pubkey, h.index),
                                 name=f"miner-{h.label}", daemon=True)
            t.start()
            self._threads.append(t)
        t = threading.Thread(target=self._watchdog, name="miner-watchdog", daemon=True)
        t.start()
        self._threads.append(t)

    def _watchdog(self) -> None:
        """Evicts a worker whose current search has run longer than watchdog_s (hung
        device) and persists the resume cursors."""
        last_save = time.time()
        while not self._stop.wait(min(1.0, self.watchdog_s / 4)):
            now = time.time()
            for h in self.alive_workers():
                if h.busy_since is not None and now - h.busy_since > self.watchdog_s:
                    self.evict(h.index, f"search hung for {now - h.busy_since:.0f}s (watchdog {self.watchdog_s:.0f}s)")
            if self.state_path and now - last_save > 5.0:
                self.save_state()
                last_save = now

    def _loop(self, backend, script_pubkey: bytes, worker: int) -> None:
        extranonce = ExtraNonce()
        h = self.health[worker]
        while not self._stop.is_set() and h.alive:
            try:
                tip = self.state.tip()
                if extranonce.prev != tip.hash:  # new tip (or first template): continue a saved sequence
                    extranonce.prev = tip.hash
                    extranonce.n = self.resume_extranonce(worker, _core.u256_hex(tip.hash))
                blk, _ = self.mine_one(script_pubkey, backend, 1 << 24, extranonce,
                                       nonce_start=self.nonce_base(worker), stop=self._stop, worker=worker)
                if blk is not None and blk.header.prev == tip.hash and h.alive:
                    st = self.state.process_new_block(blk)
                    if st.ok:
                        h.blocks += 1
                        self.metrics.inc("miner_blocks_total", 1, worker=h.label)
                    else:
                        self.metrics.inc("miner_stale_total", 1, worker=h.label)
                    log.log_print("miner", f"worker {worker} found block: {st.ok} {st.reject}")
                elif blk is not None:
                    self.metrics.inc("miner_stale_total", 1, worker=h.label)
            except Exception as e:  # keep mining; report; evict after max_failures
                self._failure(worker, e)
                time.sleep(0.05)

    def close(self) -> None:
        """Node shutdown: stop mining and end the service loop (its stop packet ends every rank)."""
        self.stop()
        if self.service is not None:
            self.service.stop()

    def stop(self) -> None:
        if self._service_req is not None:
            self.service.leader.stop_mining()
            self._service_req = None
        self._stop.set()
        for t in self._threads:
            t.join(timeout=30)
        self._threads.clear()
        self.generating = False
        if self.state_path:
            try:
                self.save_state()
            except OSError:
                pass
