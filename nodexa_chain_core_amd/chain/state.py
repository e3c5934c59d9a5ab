"""Chain state: header chain + block files + the ProcessNewBlock pipeline.

Parity (behaviour): ProcessNewBlock -> CheckBlock -> AcceptBlock ->
ActivateBestChain (src/validation.cpp:12131-12162, 12038, 11272) restricted to
what the PoW engine owns: header PoW + contextual checks (C++ HeaderChain),
structural block checks, the CLORE coinbase / community-fund rules
(C++ validation.cpp), block storage in reference-format blk?????.dat files, tip
selection by chain work, and the validation-interface signal bus
(CValidationInterface, src/validationinterface.h:37-86). UTXO/script
validation is DEFERred: non-coinbase transactions are carried
opaquely and their fees are taken as declared by the template builder.

On start-up the block index is rebuilt by scanning the blk files
(`-reindex` semantics; SURVEY S5: COMPAT-read optional).
"""
from __future__ import annotations

import os
import struct
import threading
import time
from dataclasses import dataclass, field

from .. import core
from ..utils import log, sync
from .blockindex import BlockIndexLog, scan_blk_tail
from .versionbits import VersionBits

_core = core()

REGTEST_NODEXA_KAWPOW_ACTIVATION = 1524179366 + 1  # genesis + 1: every mined regtest block is KawPow


@dataclass
class ValidationState:
    ok: bool = True
    reject: str = ""
    dos: int = 0

    @classmethod
    def invalid(cls, reason: str, dos: int = 0) -> "ValidationState":
        return cls(False, reason, dos)


class ValidationInterface:
    """Subscriber interface (CValidationInterface). Override what you need."""

    def updated_block_tip(self, tip, fork, initial_download: bool) -> None: ...

    def block_connected(self, block, index) -> None: ...

    def block_checked(self, block, state: ValidationState) -> None: ...

    def block_found(self, block_hash: bytes) -> None: ...

    def transaction_added_to_mempool(self, tx) -> None: ...


def make_params(network: str, kawpow_activation_time: int | None = None,
                equihash_activation_time: int | None = None):
    p = _core.make_chain_params(network)
    if kawpow_activation_time is not None:
        p.kawpow_activation_time = int(kawpow_activation_time)
    elif network == "regtest":
        p.kawpow_activation_time = REGTEST_NODEXA_KAWPOW_ACTIVATION
    if equihash_activation_time is not None:
        p.equihash_activation_time = int(equihash_activation_time)
    return p


@dataclass
class MempoolEntry:
    tx: object
    fee: int
    time: float = field(default_factory=time.time)
    height: int = 0          # tip height when the tx entered the pool
    fee_delta: int = 0       # prioritisetransaction adjustment (included in `fee`)
    size: int = 0            # serialized size with witness

    def vsize(self) -> int:
        base = len(self.tx.serialize(False))
        return (base * 3 + self.size + 3) // 4


MEMPOOL_DUMP_VERSION = 1


def _compact_size(n: int) -> bytes:
    if n < 0xFD:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + struct.pack("<H", n)
    if n <= 0xFFFFFFFF:
        return b"\xfe" + struct.pack("<I", n)
    return b"\xff" + struct.pack("<Q", n)


def _read_compact_size(b: bytes, off: int) -> tuple[int, int]:
    v = b[off]
    if v < 0xFD:
        return v, off + 1
    if v == 0xFD:
        return struct.unpack_from("<H", b, off + 1)[0], off + 3
    if v == 0xFE:
        return struct.unpack_from("<I", b, off + 1)[0], off + 5
    return struct.unpack_from("<Q", b, off + 1)[0], off + 9


class ChainState:
    def __init__(self, params, datadir: str | None = None, strict_height: bool = False, reindex: bool = False):
        self.params = params
        self.chain = _core.HeaderChain(params)
        self.chain.strict_kawpow_height = strict_height
        self.strict_height = strict_height
        self.lock = sync.make_lock("cs_main")
        self.cv_tip = threading.Condition(self.lock)
        self.listeners: list[ValidationInterface] = []
        self.block_pos: dict[bytes, object] = {}
        self.mempool: dict[bytes, MempoolEntry] = {}
        self.ntx: dict[bytes, int] = {}      # transactions per stored block (CBlockIndex::nTx)
        self._chain_tx: dict[bytes, int] = {}  # memo of chain_tx_count
        self.fee_stats: list[tuple[float, int]] = []  # (sat/vB, blocks to confirm) of mined pool txs
        self.mocktime = 0                     # setmocktime (0 = wall clock)
        self.block_version_override: int | None = None  # -blockversion (regtest only)
        self.transactions_updated = 0
        self.datadir = datadir
        self.store = None
        self.start_time = time.time()
        self.index_log: BlockIndexLog | None = None
        if datadir is not None:
            bdir = os.path.join(datadir, "blocks")
            os.makedirs(bdir, exist_ok=True)
            self.store = _core.BlockStore(bdir, params.message_start, params.kawpow_activation_time)
            self.index_log = BlockIndexLog(os.path.join(bdir, "index.log"))
            if reindex or not self._load_index(bdir):
                self._load_block_files()
        self.versionbits = VersionBits(self.chain, params.network_id)
        gh = self.chain.genesis().hash
        self.ntx[gh] = len(params.genesis.vtx)
        if self.store is not None and gh not in self.block_pos:
            self.block_pos[gh] = self.store.write(params.genesis)
            self.index_log.append(params.genesis.header.serialize(params.kawpow_activation_time),
                                  self.block_pos[gh], len(params.genesis.vtx))

    # ------------------------------------------------------------------ load / reindex
    def _load_block_files(self) -> None:
        """-reindex: rebuild the index from every record of the blk files, then rewrite
        blocks/index.log from the result."""
        act = self.params.kawpow_activation_time
        n, records = 0, []
        for pos, raw in self.store.scan():
            blk = _core.Block.deserialize(raw, act)
            h = self.chain.block_hash(blk.header)
            if h == self.chain.genesis().hash:
                self.block_pos[h] = pos
                records.append((blk.header.serialize(act), pos, len(blk.vtx)))
                continue
            # blocks in our files were fully validated before they were written
            r = self.chain.accept_header(blk.header, 2**62, False)
            if r.ok:
                self.block_pos[h] = pos
                self.ntx[h] = len(blk.vtx)
                records.append((blk.header.serialize(act), pos, len(blk.vtx)))
                n += 1
        self.index_log.rewrite(records)
        if n:
            log.log_printf(f"reindexed {n} blocks from block files, tip height {self.chain.height()}")

    def _load_index(self, bdir: str) -> bool:
        """LoadBlockIndex from blocks/index.log: headers accepted in one batch (no blk reads),
        then any blocks written after the last good record are recovered from the blk-file
        tail. False = no usable index (caller reindexes)."""
        act = self.params.kawpow_activation_time
        recs = self.index_log.load()
        if not recs:
            return not os.path.exists(os.path.join(bdir, "blk00000.dat"))
        hdrs = [_core.BlockHeader.deserialize(hb, act) for hb, _, _ in recs]
        res = self.chain.accept_headers(hdrs, 2**62, False)
        if len(res) != len(recs) or not all(r.ok for r in res):
            log.log_printf("block index log inconsistent with the header rules; reindexing")
            self.chain = _core.HeaderChain(self.params)
            self.chain.strict_kawpow_height = self.strict_height
            self.block_pos.clear()
            self.ntx.clear()
            return False
        last = (0, 0, 0)
        for (_, (fi, fo, fs), ntx), r in zip(recs, res):
            pos = _core.BlockPos()
            pos.file, pos.offset, pos.size = fi, fo, fs
            self.block_pos[r.index.hash] = pos
            self.ntx[r.index.hash] = ntx
            last = max(last, (fi, fo, fs))
        n = 0
        for fi, fo, raw in scan_blk_tail(bdir, bytes(self.params.message_start), last[0], last[1] + last[2]):
            blk = _core.Block.deserialize(raw, act)
            r = self.chain.accept_header(blk.header, 2**62, False)
            if not r.ok:
                break
            pos = _core.BlockPos()
            pos.file, pos.offset, pos.size = fi, fo, len(raw)
            self.block_pos[r.index.hash] = pos
            self.ntx[r.index.hash] = len(blk.vtx)
            self.index_log.append(blk.header.serialize(act), pos, len(blk.vtx))
            n += 1
        log.log_printf(f"loaded block index: {len(recs)} records (+{n} recovered from blk files), "
                       f"tip height {self.chain.height()}")
        return True

    def close(self) -> None:
        if self.index_log is not None:
            self.index_log.close()

    # ------------------------------------------------------------------ signals
    def register(self, l: ValidationInterface) -> None:
        with self.lock:
            self.listeners.append(l)

    def unregister(self, l: ValidationInterface) -> None:
        with self.lock:
            if l in self.listeners:
                self.listeners.remove(l)

    def _emit(self, name: str, *a) -> None:
        for l in list(self.listeners):
            try:
                getattr(l, name)(*a)
            except Exception as e:  # a subscriber must never break validation
                log.log_printf(f"validation listener {type(l).__name__}.{name} failed: {e}")

    # ------------------------------------------------------------------ queries
    def tip(self):
        return self.chain.tip()

    def height(self) -> int:
        return self.chain.height()

    def block_hash(self, header) -> bytes:
        return self.chain.block_hash(header)

    def get_block(self, h: bytes):
        pos = self.block_pos.get(h)
        if pos is None or self.store is None:
            return None
        return self.store.read(pos)

    def get_block_raw(self, h: bytes) -> bytes | None:
        pos = self.block_pos.get(h)
        if pos is None or self.store is None:
            return None
        return self.store.read_raw(pos)

    def adjusted_time(self) -> int:
        return int(self.mocktime or time.time())

    def arm_reorg_guard(self, peer_count: int) -> bool:
        """-maxreorg / -minreorgpeers / -minreorgage (ContextualCheckBlockHeader,
        src/validation.cpp:11815-11827): forks deeper than max_reorg_depth are rejected while the
        node has enough peers and its tip is recent. Re-armed before every P2P batch."""
        p = self.params
        armed = peer_count >= p.min_reorg_peers and (time.time() - self.tip().time) <= p.min_reorg_age
        self.chain.max_reorg_depth = p.max_reorg_depth if armed else 0
        return armed

    def chain_tx_count(self, idx) -> int:
        """CBlockIndex::nChainTx: transactions in the chain up to and including idx. Memoised per
        block hash (a stored block's count never changes), so a tip query walks back only to
        the last block already counted."""
        path = []
        while idx is not None and idx.hash not in self._chain_tx:
            path.append(idx)
            idx = self.chain.find(idx.prev_hash) if idx.height > 0 else None
        n = self._chain_tx[idx.hash] if idx is not None else 0
        complete = True  # cache only counts whose every ancestor has its data (like nChainTx != 0)
        for i in reversed(path):
            n += self.ntx.get(i.hash, 0)
            complete = complete and i.hash in self.ntx
            if complete:
                self._chain_tx[i.hash] = n
        return n

    # ------------------------------------------------------------------ mempool-lite
    def add_to_mempool(self, tx, fee: int, entry_time: float | None = None, fee_delta: int = 0) -> bytes:
        txid = tx.txid()
        with self.lock:
            new = txid not in self.mempool
            self.mempool[txid] = MempoolEntry(tx, int(fee) + int(fee_delta), entry_time or time.time(),
                                              self.chain.height(), int(fee_delta), len(tx.serialize(True)))
            self.transactions_updated += 1
        if new:
            self._emit("transaction_added_to_mempool", tx)  # TransactionAddedToMempool: P2P relay, ZMQ
        return txid

    def clear_mempool(self) -> int:
        with self.lock:
            n = len(self.mempool)
            self.mempool.clear()
            self.transactions_updated += 1
        return n

    def mempool_parents(self, txid: bytes) -> set[bytes]:
        e = self.mempool.get(txid)
        return {i.prevout.hash for i in e.tx.vin if i.prevout.hash in self.mempool} if e else set()

    def mempool_ancestors(self, txid: bytes) -> set[bytes]:
        """CalculateMemPoolAncestors over in-pool parents (txmempool.cpp)."""
        out, todo = set(), list(self.mempool_parents(txid))
        while todo:
            t = todo.pop()
            if t not in out:
                out.add(t)
                todo.extend(self.mempool_parents(t))
        return out

    def mempool_descendants(self, txid: bytes) -> set[bytes]:
        children: dict[bytes, set[bytes]] = {}
        for t in self.mempool:
            for p in self.mempool_parents(t):
                children.setdefault(p, set()).add(t)
        out, todo = set(), list(children.get(txid, ()))
        while todo:
            t = todo.pop()
            if t not in out:
                out.add(t)
                todo.extend(children.get(t, ()))
        return out

    def save_mempool(self, path: str) -> int:
        """DumpMempool (src/validation.cpp): version, count, then per tx the witness
        serialization, entry time and fee delta, then the (empty) map of deltas for txs not
        in the pool. Written to path.new and renamed."""
        with self.lock:
            entries = list(self.mempool.values())
        out = bytearray(struct.pack("<QQ", MEMPOOL_DUMP_VERSION, len(entries)))
        for e in entries:
            out += e.tx.serialize(True)
            out += struct.pack("<qq", int(e.time), int(e.fee_delta))
        out += _compact_size(0)
        tmp = path + ".new"
        with open(tmp, "wb") as f:
            f.write(out)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
        return len(entries)

    def load_mempool(self, path: str) -> int:
        """LoadMempool: re-adds every dumped tx (fees as the fee delta: no UTXO lookup)."""
        if not os.path.exists(path):
            return 0
        with open(path, "rb") as f:
            b = f.read()
        version, count = struct.unpack_from("<QQ", b, 0)
        if version != MEMPOOL_DUMP_VERSION:
            return 0
        off, n = 16, 0
        for _ in range(count):
            tx, used = _core.Transaction.deserialize_prefix(b, off)
            off += used
            t, delta = struct.unpack_from("<qq", b, off)
            off += 16
            self.add_to_mempool(tx, 0, float(t), delta)
            n += 1
        return n

    def record_confirmations(self, block, height: int) -> None:
        """Fee-estimator input (CBlockPolicyEstimator::processBlock, simplified): the feerate of
        every pool tx the block confirms and how many blocks it waited."""
        for tx in block.vtx[1:]:
            e = self.mempool.get(tx.txid())
            if e is not None:
                self.fee_stats.append((e.fee / max(1, e.vsize()), max(1, height - e.height)))
        del self.fee_stats[:-10000]

    def estimate_fee(self, target: int) -> float | None:
        """Median feerate (sat/vB) of recently mined pool txs confirmed within `target`
        blocks, or None with fewer than 10 samples (the reference's 'insufficient data')."""
        xs = sorted(f for f, waited in self.fee_stats if waited <= target)
        if len(xs) < 10:
            return None
        return xs[len(xs) // 2]

    # ------------------------------------------------------------------ ProcessNewBlock
    def check_block_header(self, header) -> ValidationState:
        r = self.chain.check_header(header, True)
        return ValidationState(r.ok, r.reject, r.dos)

    def process_new_block(self, block, check_pow: bool = True, fees_known: bool | None = None) -> ValidationState:
        """Validate + store + activate. Returns the BIP22-style state."""
        with self.lock:
            h = self.chain.block_hash(block.header)
            existing = self.chain.find(h)
            if existing is not None and h in self.block_pos:
                st = ValidationState.invalid("duplicate")
                self._emit("block_checked", block, st)
                return st
            ok, reason, dos = _core.check_block(block, self.params, True)
            if not ok:
                st = ValidationState.invalid(reason, dos)
                self._emit("block_checked", block, st)
                return st
            prev = self.chain.find(block.header.prev)
            if prev is None:
                st = ValidationState.invalid("prev-blk-not-found", 10)
                self._emit("block_checked", block, st)
                return st
            height = prev.height + 1
            ok, reason, dos = _core.contextual_check_block(block, self.params, height)
            if ok:
                fees = sum(self.mempool[tx.txid()].fee for tx in block.vtx[1:] if tx.txid() in self.mempool)
                known = (len(block.vtx) == 1) if fees_known is None else fees_known
                if not known:
                    known = all(tx.txid() in self.mempool for tx in block.vtx[1:])
                ok, reason, dos = _core.check_coinbase_rewards(block, self.params, height, fees, known)
            if not ok:
                st = ValidationState.invalid(reason, dos)
                self._emit("block_checked", block, st)
                return st
            old_tip = self.chain.tip()
            r = self.chain.accept_header(block.header, self.adjusted_time(), check_pow)
            if not r.ok:
                st = ValidationState.invalid(r.reject, r.dos)
                self._emit("block_checked", block, st)
                return st
            if self.store is not None:
                self.block_pos[h] = self.store.write(block)
                self.index_log.append(block.header.serialize(self.params.kawpow_activation_time), self.block_pos[h],
                                      len(block.vtx))
            else:
                self.block_pos[h] = None
            st = ValidationState()
            self.ntx[h] = len(block.vtx)
            self._emit("block_checked", block, st)
            self.record_confirmations(block, height)
            for tx in block.vtx[1:]:
                self.mempool.pop(tx.txid(), None)
            new_tip = self.chain.tip()
            if new_tip.hash != old_tip.hash:
                self._emit("block_connected", block, r.index)
                self._emit("updated_block_tip", new_tip, old_tip, False)
                self.cv_tip.notify_all()
                log.log_print("validation", f"new tip {_core.u256_hex(new_tip.hash)} height {new_tip.height}")
            return st

    def wait_for_tip_change(self, old_hash: bytes, timeout: float) -> bool:
        with self.cv_tip:
            return self.cv_tip.wait_for(lambda: self.chain.tip().hash != old_hash, timeout=timeout)

    # ------------------------------------------------------------------ stats
    def network_hashps(self, lookup: int = 120, height: int = -1) -> float:
        """GetNetworkHashPS (src/rpc/mining.cpp:58-93)."""
        tip = self.chain.tip()
        pb = tip
        if 0 <= height < tip.height:
            pb = self.chain.at_height(height)
        if pb is None or pb.height == 0:
            return 0.0
        interval = 2016
        if lookup <= 0:
            lookup = pb.height % interval + 1
        lookup = min(lookup, pb.height)
        min_t = max_t = pb.time
        pb0 = pb
        for _ in range(lookup):
            pb0 = self.chain.at_height(pb0.height - 1) if self.chain.in_active_chain(pb0) else self.chain.find(pb0.prev_hash)
            min_t = min(min_t, pb0.time)
            max_t = max(max_t, pb0.time)
        if min_t == max_t:
            return 0.0
        return float(pb.chain_work - pb0.chain_work) / (max_t - min_t)

