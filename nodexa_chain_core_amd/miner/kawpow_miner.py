"""KawPow mining: PoW backends and the miner controller.

Parity: generateBlocks (src/rpc/mining.cpp:117-173: template -> extranonce ->
nonce loop with CheckProofOfWork(GetHashFull) -> ProcessNewBlock),
GenerateClores / CloreMiner (src/miner.cpp:566-759: background miner threads,
nHashesPerSec for getmininginfo). Fixed here: the reference's internal miner
bumps the 32-bit nNonce, which KawPow headers do not serialize or hash
(SURVEY §3.6); this controller always searches nNonce64.

Backends
  * GpuKawpowBackend — the MI355X path: epoch DAG resident in HBM (next
    epoch prebuilt on demand), per-period JIT kernel, nonce windows of
    `intensity` nonces per launch, every share re-checked on the host.
  * CpuKawpowBackend — the reference-equivalent light-mode CPU search
    (progpow::search_light), used when no GPU is configured (e.g. regtest
    plumbing tests on CPU-only hosts).
"""
from __future__ import annotations

import threading
import time

from .. import core
from ..chain.header import from_progpow, to_progpow
from ..chain.state import ChainState
from ..utils import log
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


class GpuKawpowBackend:
    name = "gpu"

    def __init__(self, device: int = 0, intensity: int = 1 << 22):
        from ..ops.ethash import DeviceEpoch  # noqa: F401  (imports torch + _hip)

        self.device = int(device)
        self.intensity = int(intensity) // 256 * 256
        self.epochs: dict[int, object] = {}
        self.searchers: dict[int, object] = {}
        self.lock = threading.Lock()

    def _epoch(self, epoch: int):
        import torch

        from ..ops.ethash import DeviceEpoch

        if epoch not in self.epochs:
            with torch.cuda.device(self.device):
                e = DeviceEpoch(epoch, device=self.device)
                e.build()
                torch.cuda.synchronize()
                if not e.l1_matches():
                    raise RuntimeError("GPU DAG failed its L1 self-check")
            # keep at most the current and the next epoch resident
            for old in [k for k in self.epochs if k < epoch - 1]:
                self.epochs.pop(old)
                self.searchers.pop(old, None)
            self.epochs[epoch] = e
            log.log_print("gpu", f"device {self.device}: epoch {epoch} DAG {e.dag_bytes / 2**30:.2f} GiB ready")
        return self.epochs[epoch]

    def searcher(self, block_number: int):
        from ..ops.kawpow import KawpowSearcher

        epoch = block_number // _core.EPOCH_LENGTH
        with self.lock:
            ep = self._epoch(epoch)
            s = self.searchers.get(epoch)
            if s is None:
                s = KawpowSearcher(ep, block_number, prefetch_next=True)
                self.searchers[epoch] = s
            else:
                s.set_block(block_number)
            return s

    def search(self, block_number: int, header_hash: bytes, boundary: bytes, start: int, count: int):
        s = self.searcher(block_number)
        pos, end = start, start + count
        while pos < end:
            b = s.block
            n = max(b, min(self.intensity, end - pos + b - 1) // b * b)
            shares = s.search(header_hash, pos, n, boundary)
            shares = [x for x in shares if x.nonce < end]
            if shares:
                sh = shares[0]
                if not sh.verify_host(block_number, header_hash, boundary):
                    raise RuntimeError("GPU share failed host re-verification")
                return sh.nonce, sh.mix_hash, sh.final_hash
            pos += n
        return None


class MinerController:
    """generate / generatetoaddress / setgenerate on top of a PoW backend."""

    def __init__(self, state: ChainState, backends: list):
        self.state = state
        self.backends = backends
        self.hashes_done = 0
        self.hashrate = 0.0
        self._rate_t0 = time.time()
        self._threads: list[threading.Thread] = []
        self._stop = threading.Event()
        self.generating = False

    # --------------------------------------------------------------- helpers
    def _account(self, n: int) -> None:
        self.hashes_done += n
        dt = time.time() - self._rate_t0
        if dt > 4.0:
            self.hashrate = self.hashes_done / dt
            self.hashes_done = 0
            self._rate_t0 = time.time()

    def mine_one(self, script_pubkey: bytes, backend, max_tries: int, extranonce: ExtraNonce,
                 nonce_start: int = 0, stop: threading.Event | None = None):
        """Build a template and search nNonce64 in [nonce_start, +max_tries). Returns (block, tries)."""
        asm = BlockAssembler(self.state)
        tpl = asm.create_new_block(script_pubkey)
        blk = tpl.block
        extranonce.increment(blk, tpl.height)
        hdr = blk.header
        if hdr.time < self.state.params.kawpow_activation_time:
            return self._mine_legacy(blk, tpl, max_tries, nonce_start, stop)
        header_hash = to_progpow(hdr.kawpow_header_hash())
        boundary = tpl.target.to_bytes(32, "big")
        chunk = 1 << 16
        tried = 0
        while tried < max_tries and not (stop and stop.is_set()):
            n = min(chunk, max_tries - tried)
            res = backend.search(tpl.height, header_hash, boundary, nonce_start + tried, n)
            if res is None:
                tried += n
                self._account(n)
                continue
            nonce, mix, fin = res
            self._account(nonce - (nonce_start + tried) + 1)
            hdr.nonce64 = nonce
            hdr.mix_hash = from_progpow(mix)
            blk.header = hdr
            return blk, tried + (nonce - nonce_start - tried) + 1
        return None, tried

    def _mine_legacy(self, blk, tpl, max_tries: int, nonce_start: int, stop):
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
            self._account(hashes)
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
        """generateBlocks: returns the new block hashes (display hex)."""
        out: list[str] = []
        extranonce = ExtraNonce()
        backend = self.backends[0]
        while len(out) < nblocks and max_tries > 0:
            blk, tried = self.mine_one(script_pubkey, backend, max_tries, extranonce)
            max_tries -= tried
            if blk is None:
                break
            st = self.state.process_new_block(blk)
            if not st.ok:
                raise RuntimeError(f"ProcessNewBlock, block not accepted: {st.reject}")
            h = self.state.block_hash(blk.header)
            self.state._emit("block_found", h)
            out.append(_core.u256_hex(h))
        return out

    # --------------------------------------------------------------- background mining
    def set_generate(self, on: bool, script_pubkey: bytes | None = None) -> None:
        self.stop()
        if not on:
            return
        if script_pubkey is None:
            raise ValueError("setgenerate true needs -miningaddress")
        self._stop.clear()
        self.generating = True
        for i, be in enumerate(self.backends):
            t = threading.Thread(target=self._loop, args=(be, script_pubkey, i), name=f"miner-{be.name}{i}",
                                 daemon=True)
            t.start()
            self._threads.append(t)

    def _loop(self, backend, script_pubkey: bytes, worker: int) -> None:
        extranonce = ExtraNonce()
        # disjoint nNonce64 ranges per worker (the reference's miners collide on nNonce)
        base = worker << 56
        while not self._stop.is_set():
            try:
                tip = self.state.tip().hash
                blk, _ = self.mine_one(script_pubkey, backend, 1 << 24, extranonce, nonce_start=base, stop=self._stop)
                if blk is not None and blk.header.prev == tip:
                    st = self.state.process_new_block(blk)
                    log.log_print("miner", f"worker {worker} found block: {st.ok} {st.reject}")
            except Exception as e:  # keep mining; report
                log.log_printf(f"miner worker {worker} error: {e}")
                time.sleep(1.0)

    def stop(self) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=30)
        self._threads.clear()
        self.generating = False
