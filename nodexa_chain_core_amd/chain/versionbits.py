"""BIP9 version-bits deployments.

Behaviour of the reference's AbstractThresholdConditionChecker (src/versionbits.cpp:38-150):
a deployment's state is fixed per retarget-window period and computed from the last block
of the previous period (DEFINED -> STARTED once MTP >= start, STARTED -> LOCKED_IN when at
least `threshold` blocks of a period signal the bit with the 001 top bits, LOCKED_IN ->
ACTIVE one period later, DEFINED/STARTED -> FAILED once MTP >= timeout). Deployment data
per network (bit, start, timeout, per-deployment threshold / window overrides) are the
consensus constants of src/chainparams.cpp:124-153 (main), 290-319 (test), 446-475
(regtest); names and gbt_force from src/versionbits.cpp:9-37.

Used by getblocktemplate (`rules`, `vbavailable`, `vbrequired`, block version) and
getblockchaininfo (`bip9_softforks`). States are cached per (deployment, period-end hash),
so a tip query walks at most one period of headers after the first call.
"""
from __future__ import annotations

from dataclasses import dataclass

DEFINED, STARTED, LOCKED_IN, ACTIVE, FAILED = "defined", "started", "locked_in", "active", "failed"
VERSIONBITS_TOP_BITS = 0x20000000
VERSIONBITS_TOP_BITS_ASSETS = 0x30000000
VERSIONBITS_TOP_MASK = 0xE0000000


@dataclass(frozen=True)
class Deployment:
    name: str
    bit: int
    start: int
    timeout: int
    threshold: int
    window: int
    gbt_force: bool = True


def _set(start, timeout, windows):
    names = ["testdummy", "assets", "messaging_restricted", "transfer_script", "enforce_value", "coinbase"]
    bits = [28, 6, 7, 8, 9, 10]
    return [Deployment(n, b, start, timeout, th, w) for n, b, (th, w) in zip(names, bits, windows)]


_MAINNET_WINDOWS = [(1814, 2016), (1814, 2016), (1714, 2016), (1714, 2016), (1411, 2016), (1411, 2016)]
DEPLOYMENTS = {
    "main": _set(1653004800, 1653264000, _MAINNET_WINDOWS),
    "test": _set(1662998400, 1665590400, _MAINNET_WINDOWS),
    "regtest": _set(0, 999999999999, [(108, 144), (108, 144), (108, 144), (208, 288), (108, 144), (400, 500)]),
}


class VersionBits:
    def __init__(self, chain, network: str):
        self.chain = chain
        self.deployments = DEPLOYMENTS.get(network, DEPLOYMENTS["regtest"])
        self._cache: dict[tuple[str, bytes | None], str] = {}

    # ---------------------------------------------------------------- index helpers
    def _ancestor(self, idx, height: int):
        if idx is None or height < 0:
            return None
        if self.chain.in_active_chain(idx):
            return self.chain.at_height(height)
        while idx is not None and idx.height > height:
            idx = self.chain.find(idx.prev_hash)
        return idx

    def _prev(self, idx):
        return None if idx is None or idx.height == 0 else self._ancestor(idx, idx.height - 1)

    @staticmethod
    def condition(version: int, d: Deployment) -> bool:
        return (version & VERSIONBITS_TOP_MASK) == VERSIONBITS_TOP_BITS and (version >> d.bit) & 1 == 1

    # ---------------------------------------------------------------- GetStateFor
    def state_for(self, prev, d: Deployment) -> str:
        """State of the block after `prev` (prev = None for genesis)."""
        if prev is not None:
            prev = self._ancestor(prev, prev.height - ((prev.height + 1) % d.window))
        todo = []
        while (d.name, None if prev is None else prev.hash) not in self._cache:
            if prev is None:
                self._cache[(d.name, None)] = DEFINED
                break
            if prev.median_time_past() < d.start:
                self._cache[(d.name, prev.hash)] = DEFINED
                break
            todo.append(prev)
            prev = self._ancestor(prev, prev.height - d.window)
        state = self._cache[(d.name, None if prev is None else prev.hash)]
        while todo:
            prev = todo.pop()
            nxt = state
            mtp = prev.median_time_past()
            if state == DEFINED:
                if mtp >= d.timeout:
                    nxt = FAILED
                elif mtp >= d.start:
                    nxt = STARTED
            elif state == STARTED:
                if mtp >= d.timeout:
                    nxt = FAILED
                elif self._count(prev, d, d.window) >= d.threshold:
                    nxt = LOCKED_IN
            elif state == LOCKED_IN:
                nxt = ACTIVE
            self._cache[(d.name, prev.hash)] = state = nxt
        return state

    def _count(self, last, d: Deployment, n: int) -> int:
        count, idx = 0, last
        for _ in range(n):
            if idx is None:
                break
            if self.condition(idx.header.version, d):
                count += 1
            idx = self._prev(idx)
        return count

    def since_height(self, prev, d: Deployment) -> int:
        """VersionBitsTipStateSinceHeight: first height of the current state's period run."""
        state = self.state_for(prev, d)
        if state == DEFINED:
            return 0
        if prev is None:
            return 0
        prev = self._ancestor(prev, prev.height - ((prev.height + 1) % d.window))
        while True:
            earlier = self._ancestor(prev, prev.height - d.window)
            if earlier is None or self.state_for(earlier, d) != state:
                break
            prev = earlier
        return prev.height + 1

    def statistics(self, idx, d: Deployment) -> dict:
        """GetStateStatisticsFor: signalling counts in the current period up to idx."""
        end_prev = self._ancestor(idx, idx.height - ((idx.height + 1) % d.window))
        elapsed = idx.height - end_prev.height
        count = self._count(idx, d, elapsed)
        return {"period": d.window, "threshold": d.threshold, "elapsed": elapsed, "count": count,
                "possible": (d.window - d.threshold) >= (elapsed - count)}

    # ---------------------------------------------------------------- consumers
    def block_version(self, prev, assets_active: bool = True) -> int:
        """ComputeBlockVersion: top bits + every STARTED / LOCKED_IN deployment's bit."""
        v = VERSIONBITS_TOP_BITS_ASSETS if assets_active else VERSIONBITS_TOP_BITS
        for d in self.deployments:
            if self.state_for(prev, d) in (STARTED, LOCKED_IN):
                v |= 1 << d.bit
        return v

    def gbt_fields(self, prev) -> dict:
        """getblocktemplate rules / vbavailable / vbrequired (src/rpc/mining.cpp)."""
        rules, available = [], {}
        for d in self.deployments:
            st = self.state_for(prev, d)
            if st == ACTIVE:
                rules.append(d.name if d.gbt_force else "!" + d.name)
            elif st in (STARTED, LOCKED_IN):
                available[d.name] = d.bit
        return {"rules": rules, "vbavailable": available, "vbrequired": 0}

    def bip9_softforks(self, tip) -> dict:
        out = {}
        for d in self.deployments:
            st = self.state_for(tip, d)
            e = {"status": st}
            if st == STARTED:
                e["bit"] = d.bit
            e.update(startTime=d.start, timeout=d.timeout, since=self.since_height(tip, d))
            if st == STARTED:
                e["statistics"] = self.statistics(tip, d)
            out[d.name] = e
        return out
