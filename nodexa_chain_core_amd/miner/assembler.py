"""Block templates: BlockAssembler::CreateNewBlock + IncrementExtraNonce.

Parity: CreateNewBlock (src/miner.cpp:123-256): coinbase vout[0] = fees +
(100-pct)% of the subsidy to the miner script, vout[1] = subsidy*pct/100 to
the community-autonomous address, scriptSig = <height> OP_0, witness
commitment output (GenerateCoinbaseCommitment, src/validation.cpp:11779-11806)
with the 32-byte witness nonce; header: version = ComputeBlockVersion
(0x30000000 top bits | the bits of STARTED / LOCKED_IN deployments, chain/versionbits.py;
-blockversion overrides it on regtest), time = max(MTP+1, now), bits = GetNextWorkRequired, nNonce = 0,
nNonce64 = 0, nHeight = tip+1. IncrementExtraNonce (src/miner.cpp:508-525):
scriptSig = <height> <extranonce>, merkle root recomputed.

Mempool selection: addPackageTxs (src/miner.cpp:380-500) — the transaction whose package (itself
plus its not-yet-included in-pool ancestors) has the highest fee rate, with prioritisetransaction
deltas and sigop-adjusted virtual sizes, goes next, its package in parent-first order; including
a package re-scores every in-pool descendant of it (mapModifiedTx); a package that would break the
weight, -blockmaxsize or the 80000 sigop-cost limit is skipped (and selection ends after 1000
consecutive misses with the block nearly full); selection stops at the first package below
-blockmintxfee.
"""
from __future__ import annotations

import heapq

import time
from dataclasses import dataclass

from .. import core
from ..chain.state import ChainState
from ..utils import log
from ..utils.trace import traced

_core = core()

BLOCK_VERSION_ASSETS = 0x30000000
WITNESS_COMMITMENT_HEADER = bytes([0x6a, 0x24, 0xaa, 0x21, 0xa9, 0xed])


MAX_BLOCK_SIGOPS_COST = 80_000   # src/consensus/consensus.h
MAX_CONSECUTIVE_FAILURES = 1000  # addPackageTxs


class _Rate:
    """Heap key ordering packages by descending fee rate (fee / vsize, compared exactly)."""
    __slots__ = ("fee", "size")

    def __init__(self, fee: int, size: int):
        self.fee, self.size = fee, max(1, size)

    def __lt__(self, other: "_Rate") -> bool:
        return self.fee * other.size > other.fee * self.size

    def __eq__(self, other) -> bool:
        return self.fee * other.size == other.fee * self.size


@dataclass
class BlockTemplate:
    block: object          # _core.Block
    height: int
    fees: int
    coinbase_value: int
    community_value: int
    witness_commitment: bytes
    target: int
    created: float


def script_for_address(params, address: str) -> bytes:
    spk = _core.address_to_script(address, params.pubkey_prefix, params.script_prefix)
    if spk is None:
        raise ValueError(f"invalid address for {params.network_id}: {address}")
    return spk


class BlockAssembler:
    def __init__(self, state: ChainState, max_weight: int | None = None):
        self.state = state
        self.params = state.params
        # -blockmaxweight / -blockmaxsize / -blockmintxfee (BlockAssembler::Options, src/miner.cpp)
        self.max_weight = max_weight if max_weight is not None else getattr(state, "block_max_weight", 7_999_000)
        self.max_size = getattr(state, "block_max_size", None)
        self.min_fee_rate = getattr(state, "block_min_fee_rate", 0)

    @traced("miner.create_new_block")
    def create_new_block(self, script_pubkey: bytes, now: int | None = None) -> BlockTemplate:
        st = self.state
        with st.lock:
            prev = st.tip()
            height = prev.height + 1
            txs, fees = self._select_packages(st)
            subsidy = _core.block_subsidy(height)
            pct = self.params.community_autonomous_pct
            cb = _core.Transaction()
            cb.version = 1
            vin = _core.TxIn()
            vin.script_sig = _core.script_push_int(height) + b"\x00"  # CScript() << nHeight << OP_0
            cb.vin = [vin]
            miner = _core.TxOut(fees + (100 - pct) * subsidy // 100, script_pubkey)
            community = _core.TxOut(subsidy * pct // 100, script_for_address(self.params, self.params.community_autonomous_address))
            cb.vout = [miner, community]
            blk = _core.Block()
            blk.vtx = [cb] + txs
            commitment = self._add_witness_commitment(blk)
            hdr = _core.BlockHeader()
            hdr.version = st.block_version_override if st.block_version_override is not None else \
                st.versionbits.block_version(prev)  # ComputeBlockVersion (BIP9 signalling)
            hdr.prev = prev.hash
            t = int(time.time()) if now is None else int(now)
            hdr.time = max(prev.median_time_past() + 1, t)
            if hdr.time >= self.params.equihash_activation_time:
                # Equihash(200,9) extension era: the version bit selects the
                # extended header (nonce256 + solution) that consensus requires from the activation
                hdr.version = hdr.version | _core.EQUIHASH_VERSION_BIT
            hdr.height = height
            hdr.nonce = 0
            hdr.nonce64 = 0
            hdr.bits = st.chain.next_bits(hdr)
            blk.header = hdr
            root, _ = blk.merkle_root()
            hdr.merkle_root = root
            blk.header = hdr
            target, _, _ = _core.set_compact(hdr.bits)
            return BlockTemplate(blk, height, fees, miner.value, community.value, commitment, target, time.time())

    def _select_packages(self, st) -> tuple[list, int]:
        pool = st.mempool
        parents = {t: {i.prevout.hash for i in e.tx.vin if i.prevout.hash in pool} for t, e in pool.items()}
        children: dict[bytes, set] = {t: set() for t in pool}
        for t, ps in parents.items():
            for q in ps:
                children[q].add(t)
        anc: dict[bytes, frozenset] = {}
        for t in self._parents_first(pool):  # parents first: their ancestor sets are ready
            a = set(parents[t])
            for q in parents[t]:
                a |= anc[q]
            anc[t] = frozenset(a)
        stat = {}
        for t, e in pool.items():
            stripped = len(e.tx.serialize(False))
            stat[t] = (e.fee, e.vsize(), stripped * 3 + len(e.tx.serialize(True)), stripped,
                       max(0, st.mempool_sigop_cost(t)))

        in_block: set[bytes] = set()
        failed: set[bytes] = set()

        def score(t):
            pkg = [q for q in anc[t] if q not in in_block] + [t]
            return sum(stat[q][0] for q in pkg), sum(stat[q][1] for q in pkg), pkg

        heap = []

        def push(t):
            fee, vsz, _ = score(t)
            # CompareTxMemPoolEntryByAncestorFee: higher fee / size first, then the lower txid
            heapq.heappush(heap, (_Rate(fee, vsz), t, fee, vsz))

        for t in pool:
            push(t)
        txs, fees = [], 0
        weight, size, sigops = 4000, 1000, 400  # coinbase reservation (BlockAssembler::resetBlock)
        misses = 0
        while heap:
            _, t, fee, vsz = heapq.heappop(heap)
            if t in in_block or t in failed:
                continue
            cur_fee, cur_vsz, pkg = score(t)
            if (cur_fee, cur_vsz) != (fee, vsz):  # stale: an ancestor went into the block since
                push(t)
                continue
            if fee * 1000 < self.min_fee_rate * vsz:  # below -blockmintxfee: nothing better remains
                break
            pw = sum(stat[q][2] for q in pkg)
            ps = sum(stat[q][3] for q in pkg)
            pso = sum(stat[q][4] for q in pkg)
            if (weight + pw >= self.max_weight or sigops + pso >= MAX_BLOCK_SIGOPS_COST
                    or (self.max_size is not None and size + ps >= self.max_size)
                    or any(q in failed for q in pkg)):
                failed.add(t)
                misses += 1
                if misses > MAX_CONSECUTIVE_FAILURES and weight > self.max_weight - 4000:
                    break
                continue
            misses = 0
            for q in sorted(pkg, key=lambda q: (len(anc[q]), q)):  # parents before children
                if getattr(st, "print_priority", False):  # -printpriority
                    log.log_printf(f"fee {stat[q][0] * 1000 // max(1, stat[q][1])} sat/kvB txid {q[::-1].hex()}")
                txs.append(pool[q].tx)
                in_block.add(q)
                fees += stat[q][0]
            weight, size, sigops = weight + pw, size + ps, sigops + pso
            touched: set[bytes] = set()
            stack = list(pkg)
            while stack:  # UpdatePackagesForAdded: every in-pool descendant is re-scored
                for c in children[stack.pop()]:
                    if c not in touched and c not in in_block:
                        touched.add(c)
                        stack.append(c)
            for c in touched:
                if c not in failed:
                    push(c)
        return txs, fees

    @staticmethod
    def _parents_first(pool) -> list[bytes]:
        """Pool txids in arrival order, each after its in-pool parents (iterative DFS)."""
        order, seen = [], set()
        for root in list(pool):
            if root in seen:
                continue
            stack = [(root, False)]
            while stack:
                txid, expanded = stack.pop()
                if expanded:
                    order.append(txid)
                    continue
                if txid in seen:
                    continue
                seen.add(txid)
                stack.append((txid, True))
                for i in reversed(list(pool[txid].tx.vin)):
                    if i.prevout.hash in pool and i.prevout.hash not in seen:
                        stack.append((i.prevout.hash, False))
        return order

    def _add_witness_commitment(self, blk) -> bytes:
        # segwit is enabled on every network (nSegwitEnabled = true in all three params)
        cb = blk.vtx[0]
        vin = cb.vin[0]
        vin.witness = [bytes(32)]  # witness reserved value (UpdateUncommittedBlockStructures)
        cb.vin = [vin]
        vtx = [cb] + list(blk.vtx[1:])
        blk.vtx = vtx
        wroot = blk.witness_merkle_root()
        commit = _core.sha256d(wroot + bytes(32))
        spk = WITNESS_COMMITMENT_HEADER + commit
        cb.vout = list(cb.vout) + [_core.TxOut(0, spk)]
        blk.vtx = [cb] + vtx[1:]
        return spk


class ExtraNonce:
    """IncrementExtraNonce state (one per miner thread / GPU)."""

    def __init__(self):
        self.prev = None
        self.n = 0

    def increment(self, blk, height: int) -> int:
        if self.prev != blk.header.prev:
            self.n = 0
            self.prev = blk.header.prev
        self.n += 1
        vtx = list(blk.vtx)
        cb = vtx[0]
        vin = cb.vin[0]
        vin.script_sig = _core.script_push_int(height) + _core.script_push_data(_core.scriptnum(self.n))
        if len(vin.script_sig) > 100:
            raise ValueError("coinbase scriptSig too long")
        cb.vin = [vin]
        vtx[0] = cb
        blk.vtx = vtx
        hdr = blk.header
        root, _ = blk.merkle_root()
        hdr.merkle_root = root
        blk.header = hdr
        return self.n
