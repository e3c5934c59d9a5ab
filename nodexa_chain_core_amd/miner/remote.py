"""Remote-mode KawPow miner: this engine as the external GPU miner of a node.

The node side of the protocol is src/rpc/mining.cpp:722-739 and :841-932 (served here by
rpc/methods.py, and by any reference clore_blockchaind started with -miningaddress):
`getblocktemplate` carries `pprpcheader` (the KawPow header hash, hex in ProgPoW byte order),
`pprpcepoch`, `height` and `target`; the miner searches nNonce64 with ProgPoW on its GPUs and
answers `pprpcsb(header_hash, mix_hash, nonce)` with the mix in ProgPoW byte order and the
nonce as 16 hex digits. The reference keeps each header's block for 30 s and rebuilds the
template when the tip or the mempool changes, so the miner re-reads the template whenever the
previous block hash changes or `refresh` seconds have passed.

Nonce partition: worker `rank` of `world` searches nonce_base + rank * 2^56 + k, so several
processes (one per GPU) never overlap, mirroring the in-process controller's partition.
"""
from __future__ import annotations

import threading
import time

from ..utils import log


class RemoteMiner:
    def __init__(self, rpc, backend, window: int = 1 << 22, refresh: float = 15.0, rank: int = 0,
                 nonce_base: int = 0, rules=("segwit",)):
        self.rpc = rpc
        self.backend = backend
        self.window = int(window)
        self.refresh = float(refresh)
        self.rank = int(rank)
        self.nonce_base = int(nonce_base) + (self.rank << 56)
        self.rules = list(rules)
        self.stats = {"templates": 0, "windows": 0, "hashes": 0, "submitted": 0, "accepted": 0, "rejected": 0}
        self._stop = threading.Event()
        self._tpl = None
        self._tpl_time = 0.0
        self._cursor = 0

    def stop(self) -> None:
        self._stop.set()

    def template(self) -> dict:
        """The current work, re-read after `refresh` seconds or when the tip moved."""
        now = time.time()
        if self._tpl is not None and now - self._tpl_time < self.refresh:
            best = self.rpc.getbestblockhash()
            if best == self._tpl["previousblockhash"]:
                return self._tpl
        tpl = self.rpc.getblocktemplate({"rules": self.rules})
        if "pprpcheader" not in tpl:
            raise RuntimeError("the node's template has no pprpcheader (KawPow not active, or no -miningaddress)")
        if self._tpl is None or tpl["pprpcheader"] != self._tpl["pprpcheader"]:
            self._cursor = 0
        self._tpl, self._tpl_time = tpl, now
        self.stats["templates"] += 1
        return tpl

    def step(self) -> str | None:
        """One search window on the current template; submits a solution if one is found.
        Returns the pprpcsb result (None when the window had no solution)."""
        tpl = self.template()
        header_hash = bytes.fromhex(tpl["pprpcheader"])
        boundary = bytes.fromhex(tpl["target"])
        start = self.nonce_base + self._cursor
        res = self.backend.search(int(tpl["height"]), header_hash, boundary, start, self.window)
        self.stats["windows"] += 1
        if res is None:
            self._cursor += self.window
            self.stats["hashes"] += self.window
            return None
        nonce, mix, _final = res
        self.stats["hashes"] += nonce - start + 1
        self._cursor = nonce - self.nonce_base + 1
        self.stats["submitted"] += 1
        try:
            out = self.rpc.pprpcsb(tpl["pprpcheader"], bytes(mix).hex(), "%016x" % nonce)
        except RuntimeError as e:  # stale header, or a node that rejected the block
            out = str(e)
        ok = out is True or out is None or out == "duplicate"
        self.stats["accepted" if ok else "rejected"] += 1
        log.log_printf(f"remote miner: height {tpl['height']} nonce {nonce:016x} -> {out}")
        self._tpl = None  # the tip moves on an accepted block: fetch new work
        return out

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
    if a.get_bool("cpu", False):
        from .kawpow_miner import CpuKawpowBackend

        backend = CpuKawpowBackend(a.get_int("genproclimit", 1))
    else:
        from .kawpow_miner import GpuKawpowBackend

        backend = GpuKawpowBackend(a.get_int("gpu", 0), a.get_int("gpuintensity", 1 << 24))
    m = RemoteMiner(rpc, backend, window=a.get_int("minerwindow", 1 << 24), rank=a.get_int("minerrank", 0))
    blocks = a.get_int("blocks", 0)
    stats = m.run(max_blocks=blocks or None)
    print(stats)
    return 0 if stats["rejected"] == 0 else 1


if __name__ == "__main__":
    import sys

    sys.exit(main())
