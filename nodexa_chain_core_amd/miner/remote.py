"""Remote-mode miner: this engine as the external GPU miner of a node.

The node side of the protocol is src/rpc/mining.cpp:722-739 and :841-932 (served here by
rpc/methods.py, and by any reference clore_blockchaind started with -miningaddress):
`getblocktemplate` carries `pprpcheader` (the KawPow header hash, hex in ProgPoW byte order),
`pprpcepoch`, `height` and `target`; the miner searches nNonce64 with ProgPoW on its GPUs and
answers `pprpcsb(header_hash, mix_hash, nonce)` with the mix in ProgPoW byte order and the
nonce as 16 hex digits. The reference keeps each header's block for 30 s and rebuilds the
template when the tip or the mempool changes, so the miner re-reads the template whenever the
previous block hash changes or `refresh` seconds have passed. In the Equihash extension's era the
template carries `equihash.input` (the 80-byte prefix) instead, and solutions go back through
`equihashsubmit(input, nonce256, solution)`.

Nonce partition: worker `rank` of `world` searches nonce_base + rank * 2^56 + k, so several
processes (one per GPU) never overlap, mirroring the in-process controller's partition. The
search itself is the node's pipelined mining loop (miner/service.py) with a RemoteLeader.
"""
from __future__ import annotations

import threading
import time

from ..utils import log


class RemoteLeader:
    """Rank 0 of a remote miner's mining loop (miner/service.MiningService): the work packet comes
    from the node's getblocktemplate and shares go back through pprpcsb, after a full host
    re-hash. Several processes (torchrun, one per GPU) share one node connection this way: rank 0
    talks to the node, every rank searches its own nonce range."""

    def __init__(self, rpc, refresh: float = 15.0, nonce_base: int = 0, rules=("segwit",)):
        self.rpc = rpc
        self.refresh = float(refresh)
        self.nonce_base = int(nonce_base)
        self.rules = list(rules)
        self.stats = {"templates": 0, "windows": 0, "hashes": 0, "submitted": 0, "accepted": 0, "rejected": 0,
                      "bad_shares": 0}
        self.tpl = None
        self.tpl_time = 0.0
        self.job_id = 0
        self.force = False
        self.stopping = False
        self.last_result = None

    def template(self) -> dict:
        """The current work, re-read after `refresh` seconds or when the tip moved."""
        now = time.time()
        if self.tpl is not None and not self.force and now - self.tpl_time < self.refresh:
            if self.rpc.getbestblockhash() == self.tpl["previousblockhash"]:
                return self.tpl
        tpl = self.rpc.getblocktemplate({"rules": self.rules})
        if "pprpcheader" not in tpl and "equihash" not in tpl:
            raise RuntimeError("the node's template has no pprpcheader / equihash input (no -miningaddress, "
                               "or a pre-KawPow template)")
        if self.tpl is None or self._key(tpl) != self._key(self.tpl):
            self.job_id += 1
        self.tpl, self.tpl_time, self.force = tpl, now, False
        self.stats["templates"] += 1
        return tpl

    @staticmethod
    def _key(tpl: dict) -> str:
        return tpl["equihash"]["input"] if "equihash" in tpl else tpl["pprpcheader"]

    def next_work(self, repartitioned: bool = False):
        from .search import ALGO_EQUIHASH, FLAG_CLEAN, FLAG_STOP, Work

        if self.stopping:
            return Work(flags=FLAG_STOP)
        before = self.job_id
        if repartitioned:
            self.force = True
        tpl = self.template()
        flags = FLAG_CLEAN if self.job_id != before or repartitioned else 0
        if "equihash" in tpl:
            return Work(bytes.fromhex(tpl["equihash"]["input"]), bytes.fromhex(tpl["target"]), int(tpl["height"]),
                        self.job_id, self.nonce_base, flags, ALGO_EQUIHASH)
        return Work(bytes.fromhex(tpl["pprpcheader"]), bytes.fromhex(tpl["target"]), int(tpl["height"]),
                    self.job_id, self.nonce_base, flags)

    def on_results(self, records) -> None:
        from .service import _as_record

        tpl = self.tpl
        for rec in records:
            rec = _as_record(rec)
            job_id, hashes, shares = rec.job_id, rec.hashes, rec.shares
            self.stats["hashes"] += hashes
            self.stats["windows"] += hashes > 0
            if tpl is None or job_id != self.job_id or not shares:
                continue
            sh = shares[0]  # one block per template: the tip moves after it
            height = int(tpl["height"])
            if "equihash" in tpl:
                inp = tpl["equihash"]["input"]
                self.stats["submitted"] += 1
                try:
                    out = self.rpc.equihashsubmit(inp, sh.nonce256().hex(), sh.solution.hex())
                except RuntimeError as e:
                    out = str(e)
            else:
                hh = bytes.fromhex(tpl["pprpcheader"])
                if not sh.verify_full(height, hh, bytes.fromhex(tpl["target"])):
                    self.stats["bad_shares"] += 1
                    log.log_printf(f"remote miner: share nonce {sh.nonce:016x} failed the full re-hash; dropped")
                    continue
                self.stats["submitted"] += 1
                try:
                    out = self.rpc.pprpcsb(tpl["pprpcheader"], bytes(sh.mix_hash).hex(), "%016x" % sh.nonce)
                except RuntimeError as e:  # stale header, or a node that rejected the block
                    out = str(e)
            ok = out is True or out is None or out == "duplicate"
            self.stats["accepted" if ok else "rejected"] += 1
            self.last_result = out
            log.log_printf(f"remote miner: height {height} nonce {sh.nonce:016x} -> {out}")
            self.force = True  # the tip moves on an accepted block: fetch new work
            tpl = None

    def shutdown(self) -> None:
        self.stopping = True


def _device_for(backend):
    """A miner/search device for `backend`: a search device as is; None means this host's CPU."""
    from .search import CpuSearchDevice

    if backend is not None and hasattr(backend, "submit") and hasattr(backend, "wait"):
        return backend
    return CpuSearchDevice()


class RemoteMiner:
    """The remote-mode miner: the node's own mining loop (pipelined windows, device-side stale-work
    abort, full share re-hash) with a RemoteLeader in place of the chain.

    Nonce partition: worker `rank` of an external set of miners searches nonce_base + rank * 2^56
    + k (inside one torchrun world the service adds its own rank the same way)."""

    def __init__(self, rpc, backend, window: int = 1 << 22, refresh: float = 15.0, rank: int = 0,
                 nonce_base: int = 0, rules=("segwit",)):
        from .service import MiningService

        self.rpc = rpc
        self.rank = int(rank)
        self.leader = RemoteLeader(rpc, refresh, int(nonce_base) + (self.rank << 56), rules)
        self.dev = _device_for(backend)
        if getattr(self.dev, "name", "") == "cpu" and hasattr(self.dev, "max_window"):
            self.dev.max_window = min(self.dev.max_window, int(window))
        self.service = MiningService(self.dev, self.leader, window=int(window))
        self.stats = self.leader.stats
        self._stop = threading.Event()

    def stop(self) -> None:
        self._stop.set()

    def template(self) -> dict:
        return self.leader.template()

    def step(self) -> str | None:
        """One iteration of the loop; returns the pprpcsb result of a share submitted in it."""
        self.leader.last_result = None
        self.service.step()
        return self.leader.last_result

    def run(self, max_blocks: int | None = None, max_seconds: float | None = None) -> dict:
        t0 = time.time()
        while not self._stop.is_set():
            if max_blocks is not None and self.stats["accepted"] >= max_blocks:
                break
            if max_seconds is not None and time.time() - t0 > max_seconds:
                break
            try:
                self.step()
            except (OSError, ConnectionError) as e:
                log.log_printf(f"remote miner: node unreachable ({e}); retrying")
                self._stop.wait(1.0)
        try:
            self.service.pipe.drain()
        except Exception:  # noqa: BLE001
            pass
        self.stats["seconds"] = round(time.time() - t0, 3)
        return dict(self.stats)


def main(argv: list[str] | None = None) -> int:
    """nodexa-miner: -rpcconnect / -rpcport / -rpcuser / -rpcpassword of the node, -gpus=0,1..
    (one process per GPU: pass -minerrank), -cpu for the host backend, -blocks=N to stop after N."""
    import sys

    from ..chain.state import make_params
    from ..rpc.client import RPCClient
    from ..utils.config import ArgsManager

    a = ArgsManager()
    a.parse_parameters(sys.argv[1:] if argv is None else argv)
    params = make_params(a.network)
    rpc = RPCClient(a.get("rpcconnect", "127.0.0.1"), a.get_int("rpcport", params.default_rpc_port),
                    a.get("rpcuser"), a.get("rpcpassword"), None, timeout=60.0)
    from .service import make_rank_device

    cpu = a.get_bool("cpu", False)
    backend = make_rank_device(cpu, None if cpu else a.get_int("gpu", 0), window=a.get_int("minerwindow", 4096))
    m = RemoteMiner(rpc, backend, window=a.get_int("minerwindow", 1 << 25), rank=a.get_int("minerrank", 0))
    blocks = a.get_int("blocks", 0)
    stats = m.run(max_blocks=blocks or None)
    print(stats)
    return 0 if stats["rejected"] == 0 else 1


if __name__ == "__main__":
    import sys

    sys.exit(main())
