"""Chain state: header chain, block and undo files, the UTXO set and the ProcessNewBlock pipeline.

Parity (behaviour): ProcessNewBlock -> CheckBlock -> AcceptBlock -> ActivateBestChain ->
ConnectTip / DisconnectTip -> ConnectBlock / DisconnectBlock (src/validation.cpp:12131-12162,
12038, 11272, 10958, 10052, 9479): header PoW + contextual checks (C++ HeaderChain), structural
block checks, block storage in reference-format blk?????.dat files, tip selection by chain work,
then the UTXO set (C++ CoinsView, chain/coins.hpp) follows the best header chain: every block is
connected with its inputs, sequence locks, sigop cost and scripts checked, the CLORE coinbase /
community-fund rules applied to the real fees, and undo data written to rev?????.dat
(chain/undo.py) so a reorg can disconnect. AcceptToMemoryPool checks transactions against the
same UTXO set. The validation-interface signal bus is CValidationInterface
(src/validationinterface.h:37-86).

Signatures in blocks are verified in one GPU batch per block when a GPU is present
(ops/secp.verify_batch; the reference spreads them over its CCheckQueue CPU threads). The batch
result is only trusted where it cannot differ from the reference: any input whose signature the
batch rejects is re-run on the host, and a block whose deferred run fails is re-connected with
host checks (`_connect_one`).

Storage (-dbformat, `detect_db_format`): by default the block index and the UTXO set live in
LevelDB-format stores with the reference's keys — blocks/index/ (BlockTreeDB: 'b' CDiskBlockIndex
records, 'f' file infos, 'l', 'R') and chainstate/ (CCoinsViewDB: 'C' coins, 'B' best block),
values obfuscated as CDBWrapper does (csrc/store/) — so a reference datadir opens here without
-reindex and ours opens in the reference. A flush — every `flush_interval` connected blocks and at
shutdown — writes only the outputs added or spent since the previous flush plus 'B' as one synced
batch (CCoinsViewDB::BatchWrite, src/txdb.cpp:91-), so its cost follows the blocks connected, not
the size of the UTXO set. The older "journal" layout (chainstate/coins.dat snapshot + coins.log
journal, blocks/index.log) is still read and written for datadirs that hold it. On start-up
blocks stored past the UTXO set's best block are reconnected (ReplayBlocks-lite), and a state
whose best block is unknown, or whose last flush did not complete, is rebuilt from genesis.
"""
from __future__ import annotations

import os
import random
import struct
import threading
import time
from dataclasses import dataclass, field

from .. import core
from ..utils import log, sync
from . import policy
from .blockindex import BLOCK_FAILED_VALID, BLOCK_HAVE_DATA, BLOCK_HAVE_UNDO, BlockIndexLog, BlockTreeDB, scan_blk_tail
from .undo import UndoStore
from .versionbits import VersionBits

_core = core()

# -kawpowactivationtime value that makes every mined regtest block KawPow (genesis time + 1). The
# regtest default is the reference's own (3582830167, src/chainparams.cpp:566-570: X16RV2 mining);
# KawPow regtest is an explicit override, never the default
REGTEST_KAWPOW_FROM_GENESIS = 1524179366 + 1


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

    # ConnectTip / DisconnectTip post-processing, called synchronously (under the chain lock) for
    # each block as it joins or leaves the UTXO set, with that block's undo data (the coins it
    # spent): the asset-messaging and reward-snapshot hooks of src/validation.cpp:10517, 11058
    def connect_tip(self, block, index, undo: bytes) -> None: ...

    def disconnect_tip(self, block, index, undo: bytes) -> None: ...

    def new_asset_message(self, message) -> None: ...


DB_FORMATS = ("leveldb", "journal")
# chainstate/ record: the height at which a reference datadir's assets/ databases were imported
ASSETS_IMPORT_KEY = b"\x02assets.import"


def detect_db_format(datadir: str | None, requested: str | None = None) -> str:
    """Storage layout of a datadir (-dbformat):

    "leveldb"  blocks/index/ and chainstate/ as LevelDB-format stores in the reference's key
               layout (BlockTreeDB, CCoinsViewDB): reference datadirs open without -reindex and
               ours open in the reference. The default for new datadirs.
    "journal"  blocks/index.log plus chainstate/coins.dat + coins.log (this engine's earlier
               layout); existing datadirs of that layout keep it unless another is requested.
    Requesting a format a datadir does not hold migrates it: the block index is rebuilt from the
    blk files (-reindex) and the UTXO set replayed from the stored blocks.
    """
    if requested:
        if requested not in DB_FORMATS:
            raise ValueError(f"-dbformat must be one of {', '.join(DB_FORMATS)}")
        return requested
    if datadir is None:
        return "memory"
    if os.path.exists(os.path.join(datadir, "blocks", "index", "CURRENT")):
        return "leveldb"
    if any(os.path.exists(os.path.join(datadir, *p)) for p in (("blocks", "index.log"), ("chainstate", "coins.dat"),
                                                               ("chainstate", "coins.log"))):
        return "journal"
    return "leveldb"


def make_params(network: str, kawpow_activation_time: int | None = None,
                equihash_activation_time: int | None = None):
    p = _core.make_chain_params(network)
    if kawpow_activation_time is not None:
        p.kawpow_activation_time = int(kawpow_activation_time)
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
    sigop_cost: int = -1     # GetTransactionSigOpCost (-1: not computed, e.g. loaded from mempool.dat)
    bytes_per_sigop: int = 20  # -bytespersigop in force when the entry was made
    _weight: int = field(default=-1, repr=False, compare=False)

    def vsize(self) -> int:
        """GetTxSize = GetVirtualTransactionSize(weight, sigop cost) (src/policy/policy.cpp): a
        transaction heavy in signature operations counts as bytes_per_sigop bytes per sigop."""
        if self._weight < 0:
            self._weight = len(self.tx.serialize(False)) * 3 + self.size
        return (max(self._weight, max(0, self.sigop_cost) * self.bytes_per_sigop) + 3) // 4


MEMPOOL_DUMP_VERSION = 1
DEFAULT_MIN_RELAY_TX_FEE = 1_000_000   # sat per kvB (src/validation.h:69)
DEFAULT_INCREMENTAL_RELAY_FEE = 1000   # sat per kvB (src/policy/policy.h:36)
DEFAULT_ENABLE_REPLACEMENT = False     # -mempoolreplacement (src/validation.h:163)
MAX_STANDARD_TX_WEIGHT = 400_000       # src/policy/policy.h:28
DEFAULT_BYTES_PER_SIGOP = 20           # -bytespersigop (src/policy/policy.h)
MIN_BLOCKS_TO_KEEP = 288              # blocks below the tip never pruned (src/validation.h:240)
MIN_DISK_SPACE_FOR_BLOCK_FILES = 550 << 20  # smallest -prune target (src/validation.h:253)
PRUNE_AFTER_HEIGHT = {"main": 100_000, "test": 1000, "regtest": 1000}  # nPruneAfterHeight
BLOCKFILE_CHUNK_SIZE, UNDOFILE_CHUNK_SIZE = 16 << 20, 1 << 20  # headroom FindFilesToPrune keeps
COIN_CACHE_ENTRY_BYTES = 128           # memory of one pending UTXO change (entry + map node), for -dbcache
MAX_STANDARD_TX_SIGOPS_COST = 80_000 // 5  # MAX_BLOCK_SIGOPS_COST / 5 (src/policy/policy.h)
MAX_FEE_ESTIMATION_TIP_AGE = 3 * 60 * 60  # src/validation.h (IsCurrentForFeeEstimation)
# package and expiry limits (src/validation.h:77-85) and the raw-tx fee cap (DEFAULT_TRANSACTION_MAXFEE)
DEFAULT_ANCESTOR_LIMIT, DEFAULT_ANCESTOR_SIZE_LIMIT = 200, 250        # count, kvB
DEFAULT_DESCENDANT_LIMIT, DEFAULT_DESCENDANT_SIZE_LIMIT = 200, 250
DEFAULT_MEMPOOL_EXPIRY = 336                                          # hours
DEFAULT_TRANSACTION_MAXFEE = 1000 * 100_000_000
DEFAULT_BLOCK_MIN_TX_FEE = 1000                                       # sat per kvB (src/policy/policy.h:26)
DEFAULT_MAX_TIP_AGE = 24 * 60 * 60                                    # -maxtipage (src/validation.h)
DEFAULT_MAX_MEMPOOL_SIZE = 300                                        # -maxmempool, MB (src/policy/policy.h:34)
ROLLING_FEE_HALFLIFE = 60 * 60 * 12                                   # src/txmempool.h
MEMPOOL_ENTRY_OVERHEAD = 320  # bytes of bookkeeping per entry counted by mempool_usage (DynamicMemoryUsage analogue)
MAX_STANDARD_SCRIPTSIG_SIZE = 1650
GPU_SIG_BATCH_MIN = 16                 # below this many signatures a block is checked on the host


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
    def __init__(self, params, datadir: str | None = None, strict_height: bool = False, reindex: bool = False,
                 indexes: dict | None = None, db_format: str | None = None, reindex_chainstate: bool = False):
        """`reindex`: rebuild the block index from the blk files (and the chain state with it);
        `reindex_chainstate`: keep the block index, rebuild the UTXO set, asset state and indexes by
        connecting the stored blocks again from genesis (-reindex-chainstate, src/init.cpp:1500)."""
        self.params = params
        self.reindex_chainstate = reindex_chainstate
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
        self.fee_estimator = _core.FeeEstimator()  # CBlockPolicyEstimator (csrc/chain/fees.cpp)
        self.mocktime = 0                     # setmocktime (0 = wall clock)
        self.block_version_override: int | None = None  # -blockversion (regtest only)
        self.transactions_updated = 0
        self.datadir = datadir
        self.assets_import_height = -1  # see _import_reference_assets
        self.store = None
        self.start_time = time.time()
        self.index_log: BlockIndexLog | None = None
        self._mem_blocks: dict[bytes, object] = {}  # block data when there is no datadir
        self.min_relay_fee = DEFAULT_MIN_RELAY_TX_FEE
        self.incremental_relay_fee = DEFAULT_INCREMENTAL_RELAY_FEE  # -incrementalrelayfee
        self.enable_replacement = DEFAULT_ENABLE_REPLACEMENT       # -mempoolreplacement
        self.require_standard = params.network_id == "main"        # fRequireStandard / -acceptnonstdtxn
        self.datacarrier, self.datacarrier_size = True, policy.MAX_OP_RETURN_RELAY  # -datacarrier[size]
        self.permit_bare_multisig = True                            # -permitbaremultisig
        self.dust_relay_fee = policy.DUST_RELAY_TX_FEE              # -dustrelayfee
        self.ancestor_limits = (DEFAULT_ANCESTOR_LIMIT, DEFAULT_ANCESTOR_SIZE_LIMIT * 1000)        # -limitancestor*
        self.descendant_limits = (DEFAULT_DESCENDANT_LIMIT, DEFAULT_DESCENDANT_SIZE_LIMIT * 1000)  # -limitdescendant*
        self.mempool_expiry = DEFAULT_MEMPOOL_EXPIRY * 3600         # -mempoolexpiry (seconds)
        self.max_tx_fee = DEFAULT_TRANSACTION_MAXFEE                # -maxtxfee (absurd-fee cap)
        self.bytes_per_sigop = DEFAULT_BYTES_PER_SIGOP              # -bytespersigop
        self.last_replaced: list = []  # transactions the last accepted replacement pushed out
        self.block_max_weight = 7_999_000                           # -blockmaxweight
        self.block_max_size: int | None = None                      # -blockmaxsize
        self.block_min_fee_rate = DEFAULT_BLOCK_MIN_TX_FEE          # -blockmintxfee
        self.assume_valid: bytes | None = None                      # -assumevalid (block hash, storage order)
        self.minimum_chain_work = 0                                 # -minimumchainwork
        self.max_tip_age = DEFAULT_MAX_TIP_AGE                      # -maxtipage
        self.importing = False                                      # -loadblock / -reindex in progress
        self._ibd_latched = False
        self.scripts_skipped = 0                                    # blocks connected under -assumevalid
        self.db_crash_ratio = 0                                     # -dbcrashratio fault injection
        self.check_block_index_enabled = False                      # -checkblockindex
        self.max_mempool_bytes = DEFAULT_MAX_MEMPOOL_SIZE * 1_000_000  # -maxmempool
        self.rolling_min_fee = 0.0       # rollingMinimumFeeRate (sat per kvB)
        self._last_rolling_update = 0.0
        self._block_since_bump = False
        self.script_threads = min(16, os.cpu_count() or 1)  # -par: script-check threads (CCheckQueue)
        self.gpu_signatures = "auto"          # "auto" (GPU when present), "on" or "off" (-gpusigs)
        self.flush_interval = 1000
        self.coins_cache_bytes = 450 << 20     # -dbcache: flush once the pending UTXO changes pass it
        self.prune_target = 0                  # -prune: 0 off, 1 manual (pruneblockchain), else bytes
        self.prune_after_height = PRUNE_AFTER_HEIGHT.get(params.network_id, 1000)
        self._check_for_pruning = False
        self.journal_compact_bytes = 64 << 20  # fold coins.log into coins.dat past this size (or the snapshot's)
        self._since_flush = 0
        self.sig_stats = {"gpu_batches": 0, "gpu_sigs": 0, "host_rechecks": 0}
        self.db_format = detect_db_format(datadir, db_format)
        self.coins_db = None
        self._coins_obf = b""
        if datadir is not None:
            bdir = os.path.join(datadir, "blocks")
            os.makedirs(bdir, exist_ok=True)
            self.store = _core.BlockStore(bdir, params.message_start, params.kawpow_activation_time)
            if self.db_format == "leveldb":
                self.index_log = BlockTreeDB(os.path.join(bdir, "index"), params.kawpow_activation_time)
                reindex = reindex or self.index_log.reindexing()  # an interrupted -reindex resumes
            else:
                self.index_log = BlockIndexLog(os.path.join(bdir, "index.log"))
            if reindex or not self._load_index(bdir):
                self._load_block_files()
        self.versionbits = VersionBits(self.chain, params.network_id)
        gh = self.chain.genesis().hash
        self.ntx[gh] = len(params.genesis.vtx)
        if self.store is not None and gh not in self.block_pos:
            self.block_pos[gh] = self.store.write(params.genesis)
            self.index_log.append(params.genesis.header.serialize(params.kawpow_activation_time),
                                  self.block_pos[gh], len(params.genesis.vtx), height=0, block_hash=gh,
                                  time=params.genesis.header.time)
        bdir = os.path.join(datadir, "blocks") if datadir else None
        self.undo = UndoStore(bdir, bytes(params.message_start))
        for h, fi, upos in getattr(self, "_undo_adopt", ()):  # undo records a reference index located
            if h not in self.undo.pos and not self.undo.adopt(h, fi, upos):
                log.log_printf(f"undo record of {_core.u256_hex(h)} not found at rev{fi:05d}:{upos}")
        self._undo_adopt = []
        if self.db_format == "leveldb" and self.index_log is not None:
            # records rebuilt by a reindex carry no undo position yet: take them from the undo store
            for h, e in list(self.index_log.entries.items()):
                u = self.undo.pos.get(h)
                if u is not None and not e[1] & BLOCK_HAVE_UNDO and u[0] == e[3]:
                    self.index_log.set_undo(h, u[0], u[1], u[2])
        self.asset_undo = UndoStore(bdir, bytes(params.message_start), prefix="aun")
        self.coins_path = os.path.join(datadir, "chainstate", "coins.dat") if datadir else None
        self.coins_log = os.path.join(datadir, "chainstate", "coins.log") if datadir else None
        self.assets_path = os.path.join(datadir, "chainstate", "assets.dat") if datadir else None
        self.indexes_path = os.path.join(datadir, "chainstate", "indexes.dat") if datadir else None
        self.index_flags = dict(indexes or {})  # txindex / addressindex / spentindex / timestampindex
        self._stored_index_flags = {}
        if self.db_format == "leveldb" and self.index_log is not None:
            for k, v in self.index_flags.items():  # WriteFlag (src/init.cpp), read back by the reference
                self._stored_index_flags[k] = self.index_log.flag(k)
                if self._stored_index_flags[k] != bool(v):
                    self.index_log.set_flag(k, bool(v))
        self.coins = _core.CoinsView()
        self.assets = _core.AssetsState()
        self.indexes = self._new_indexes()
        self._init_coins()

    def _new_indexes(self):
        ix = _core.ChainIndexes(**self.index_flags)
        # blocks/index keeps the indexes as records (CBlockTreeDB layout): connect / disconnect
        # journal their changes for the next flush
        ix.journal = self.db_format == "leveldb" and self.index_log is not None and any(self.index_flags.values())
        return ix

    # ------------------------------------------------------------------ load / reindex
    def _load_block_files(self) -> None:
        """-reindex: rebuild the index from every record of the blk files, then rewrite
        blocks/index.log from the result."""
        act = self.params.kawpow_activation_time
        if self.db_format == "leveldb":
            self.index_log.set_reindexing(True)  # DB_REINDEX_FLAG: an interrupted reindex restarts
        n, records = 0, []
        for pos, raw in self.store.scan():
            blk = _core.Block.deserialize(raw, act)
            h = self.chain.block_hash(blk.header)
            if h == self.chain.genesis().hash:
                self.block_pos[h] = pos
                records.append((blk.header.serialize(act), pos, len(blk.vtx), 0, h, blk.header.time))
                continue
            # blocks in our files were fully validated before they were written
            r = self.chain.accept_header(blk.header, 2**62, False)
            if r.ok:
                self.block_pos[h] = pos
                self.ntx[h] = len(blk.vtx)
                records.append((blk.header.serialize(act), pos, len(blk.vtx), r.index.height, h, blk.header.time))
                n += 1
        self.index_log.rewrite(records)
        if self.db_format == "leveldb":
            self.index_log.set_reindexing(False)
        if n:
            log.log_printf(f"reindexed {n} blocks from block files, tip height {self.chain.height()}")

    def _load_index(self, bdir: str) -> bool:
        """LoadBlockIndex from blocks/index.log: headers accepted in one batch (no blk reads),
        then any blocks written after the last good record are recovered from the blk-file
        tail. False = no usable index (caller reindexes)."""
        act = self.params.kawpow_activation_time
        if self.db_format == "leveldb":
            return self._load_block_tree(bdir)
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

    def _load_block_tree(self, bdir: str) -> bool:
        """LoadBlockIndexGuts from blocks/index/ in the reference's LevelDB layout
        (src/txdb.cpp:230-260, validation.cpp LoadBlockIndexDB): every 'b' record's header is
        accepted in height order in one batch (header-only entries included), stored blocks and
        their undo records are located from the records, failed blocks are marked again, and
        blocks written to the blk files after the last record are recovered from the file tail.
        False = no usable index (the caller reindexes)."""
        act = self.params.kawpow_activation_time
        try:
            recs = self.index_log.load()
        except IOError as e:
            log.log_printf(f"{e}; reindexing")
            return False
        if not recs:
            return not os.path.exists(os.path.join(bdir, "blk00000.dat"))
        hdrs = [_core.BlockHeader.deserialize(r[7], act) for r in recs]
        res = self.chain.accept_headers(hdrs, 2**62, False)
        if len(res) != len(recs) or not all(r.ok for r in res):
            log.log_printf("block index records inconsistent with the header rules; reindexing")
            self.chain = _core.HeaderChain(self.params)
            self.chain.strict_kawpow_height = self.strict_height
            self.block_pos.clear()
            self.ntx.clear()
            return False
        fds: dict[int, int] = {}
        last, failed, n_data = (0, 0, 0), [], 0
        self._undo_adopt = []
        try:
            for (h, height, status, ntx, fi, dpos, upos, hb), r in zip(recs, res):
                if status & BLOCK_HAVE_DATA:
                    fd = fds.get(fi)
                    if fd is None:
                        fd = fds[fi] = os.open(self.store.path(fi), os.O_RDONLY)
                    frame = os.pread(fd, 8, dpos - 8)
                    if len(frame) != 8 or frame[:4] != bytes(self.params.message_start):
                        log.log_printf(f"block {_core.u256_hex(h)} missing at blk{fi:05d}:{dpos}; reindexing")
                        return False
                    pos = _core.BlockPos()
                    pos.file, pos.offset, pos.size = fi, dpos, struct.unpack("<I", frame[4:])[0]
                    self.block_pos[r.index.hash] = pos
                    last = max(last, (fi, dpos, pos.size))
                    n_data += 1
                if ntx:  # nTx stays with a pruned block's header
                    self.ntx[r.index.hash] = ntx
                if status & BLOCK_HAVE_UNDO:
                    self._undo_adopt.append((h, fi, upos))
                if status & BLOCK_FAILED_VALID:
                    failed.append(h)
        except OSError as e:
            log.log_printf(f"cannot read the blk files the block index names ({e}); reindexing")
            return False
        finally:
            for fd in fds.values():
                os.close(fd)
        for h in failed:
            self.chain.invalidate(h)
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
            self.index_log.append(blk.header.serialize(act), pos, len(blk.vtx), height=r.index.height,
                                  block_hash=r.index.hash, time=blk.header.time)
            n += 1
        log.log_printf(f"loaded block index (LevelDB): {len(recs)} records, {n_data} with data "
                       f"(+{n} recovered from blk files), tip height {self.chain.height()}")
        return True

    def close(self) -> None:
        self.flush()
        if self.index_log is not None:
            self.index_log.close()
        self.undo.close()
        self.asset_undo.close()
        if self.coins_db is not None:
            self.coins_db.close()
            self.coins_db = None

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
            fn = getattr(l, name, None)
            if fn is None:  # listeners need not implement every hook
                continue
            try:
                fn(*a)
            except Exception as e:  # a subscriber must never break validation
                log.log_printf(f"validation listener {type(l).__name__}.{name} failed: {e}")

    # ------------------------------------------------------------------ queries
    def tip(self):
        """chainActive.Tip(): the last block connected to the UTXO set (the header chain may run
        ahead of it while block data is still being fetched)."""
        return self.coins_tip() if hasattr(self, "coins") else self.chain.tip()

    def height(self) -> int:
        return self.tip().height

    def block_hash(self, header) -> bytes:
        return self.chain.block_hash(header)

    def get_block(self, h: bytes):
        if self.store is None:
            return self._mem_blocks.get(h)
        pos = self.block_pos.get(h)
        if pos is None:
            return None
        return self.store.read(pos)

    def get_block_raw(self, h: bytes) -> bytes | None:
        if self.store is None:
            blk = self._mem_blocks.get(h)
            return None if blk is None else blk.serialize(self.params.kawpow_activation_time)
        pos = self.block_pos.get(h)
        if pos is None:
            return None
        return self.store.read_raw(pos)

    def adjusted_time(self) -> int:
        """GetAdjustedTime: the clock (or setmocktime) plus the peers' median offset (timedata)."""
        return int(self.mocktime or time.time()) + getattr(self, "time_offset", 0)

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
    def add_to_mempool(self, tx, fee: int, entry_time: float | None = None, fee_delta: int = 0,
                       replacement: bool = False, sigop_cost: int = -1) -> bytes:
        txid = tx.txid()
        with self.lock:
            new = txid not in self.mempool
            e = MempoolEntry(tx, int(fee) + int(fee_delta), entry_time or self.adjusted_time(),  # GetTime(): mocktime aware
                             self.chain.height(), int(fee_delta), len(tx.serialize(True)), int(sigop_cost),
                             self.bytes_per_sigop)
            if new:
                # processTransaction: fee estimates only learn from a node that is current, and not
                # from replacements or children of pool transactions (validFeeEstimate)
                valid = (not replacement and self.is_current_for_fee_estimation()
                         and not any(i.prevout.hash in self.mempool for i in tx.vin))
                tip = self.coins_tip()
                self.fee_estimator.process_tx(txid, tip.height, int(fee), e.vsize(), valid)
            self.mempool[txid] = e
            self.transactions_updated += 1
        if new:
            self._emit("transaction_added_to_mempool", tx)  # TransactionAddedToMempool: P2P relay, ZMQ
        return txid

    def mempool_usage(self) -> int:
        """DynamicMemoryUsage analogue: serialized sizes plus a fixed per-entry overhead."""
        return sum(e.size + MEMPOOL_ENTRY_OVERHEAD for e in self.mempool.values())

    def mempool_min_fee(self) -> int:
        """CTxMemPool::GetMinFee (sat per kvB): the rolling floor left by TrimToSize, decaying
        with a 12 h half-life (3 h / 6 h while the pool is under a quarter / half full) once a
        block has arrived since the last bump; 0 below half the incremental relay fee."""
        if not self._block_since_bump or self.rolling_min_fee == 0:
            return int(round(self.rolling_min_fee))
        now = self.adjusted_time()
        if now > self._last_rolling_update + 10:
            half, usage = ROLLING_FEE_HALFLIFE, self.mempool_usage()
            if usage < self.max_mempool_bytes / 4:
                half /= 4
            elif usage < self.max_mempool_bytes / 2:
                half /= 2
            self.rolling_min_fee /= 2.0 ** ((now - self._last_rolling_update) / half)
            self._last_rolling_update = now
            if self.rolling_min_fee < self.incremental_relay_fee / 2:
                self.rolling_min_fee = 0.0
                return 0
        return max(int(round(self.rolling_min_fee)), self.incremental_relay_fee)

    def trim_mempool(self) -> int:
        """TrimToSize: while over -maxmempool, evict the package (an entry and its descendants)
        with the lowest descendant feerate and raise the rolling floor to that feerate plus the
        incremental relay fee."""
        gone = 0
        with self.lock:
            while self.mempool and self.mempool_usage() > self.max_mempool_bytes:
                best = None
                for t, e in self.mempool.items():
                    desc = self.mempool_descendants(t)
                    fee = e.fee + sum(self.mempool[d].fee for d in desc)
                    size = e.vsize() + sum(self.mempool[d].vsize() for d in desc)
                    score = fee * 1000 / max(1, size)
                    if best is None or score < best[0]:
                        best = (score, t, desc)
                score, t, desc = best
                rate = score + self.incremental_relay_fee
                if rate > self.rolling_min_fee:  # trackPackageRemoved
                    self.rolling_min_fee = rate
                    self._block_since_bump = False
                for x in {t} | desc:
                    self.pool_remove(x)
                    gone += 1
            if gone:
                self.transactions_updated += 1
        return gone

    def pool_remove(self, txid: bytes, in_block: bool = False) -> None:
        """removeUnchecked: drop a pool entry and stop tracking it for fee estimation (an entry
        that leaves unconfirmed counts as a failure at its feerate)."""
        if self.mempool.pop(txid, None) is not None:
            self.fee_estimator.remove_tx(txid, in_block)

    def is_initial_block_download(self) -> bool:
        """IsInitialBlockDownload (src/validation.cpp): importing, a tip with less work than
        -minimumchainwork, or a tip older than -maxtipage; once false it stays false (latched)."""
        if self._ibd_latched:
            return False
        tip = self.coins_tip()
        if self.importing or tip is None or tip.chain_work < self.minimum_chain_work:
            return True
        if tip.time < self.adjusted_time() - self.max_tip_age:
            return True
        self._ibd_latched = True
        return False

    def _assumed_valid(self, idx) -> bool:
        """ConnectBlock's fScriptChecks = false: `idx` is an ancestor of the -assumevalid block and
        of the best header, and the best header has at least -minimumchainwork."""
        if self.assume_valid is None:
            return False
        av = self.chain.find(self.assume_valid)
        if av is None or av.height < idx.height:
            return False
        best = self.chain.tip()
        if best.chain_work < self.minimum_chain_work:
            return False

        def ancestor(i, h):
            while i is not None and i.height > h:
                i = self.chain.find(i.prev_hash)
            return i

        a1, a2 = ancestor(av, idx.height), ancestor(best, idx.height)
        return a1 is not None and a2 is not None and a1.hash == idx.hash and a2.hash == idx.hash

    def is_current_for_fee_estimation(self) -> bool:
        """IsCurrentForFeeEstimation (src/validation.cpp): the tip is under 3 hours old and
        within one block of the best header."""
        tip = self.coins_tip()
        if tip is None or tip.time < self.adjusted_time() - MAX_FEE_ESTIMATION_TIP_AGE:
            return False
        return tip.height >= self.chain.height() - 1

    def save_fee_estimates(self, path: str) -> None:
        """Shutdown: FlushUnconfirmed (every tracked pool entry counts as unconfirmed), then
        fee_estimates.dat in the reference's format, written to path.new and renamed."""
        self.fee_estimator.flush_unconfirmed()
        tmp = path + ".new"
        with open(tmp, "wb") as f:
            f.write(self.fee_estimator.serialize())
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)

    def load_fee_estimates(self, path: str) -> bool:
        if not os.path.exists(path):
            return False
        with open(path, "rb") as f:
            ok, err = self.fee_estimator.deserialize(f.read())
        if not ok:
            log.log_printf(f"CBlockPolicyEstimator::Read(): unable to read policy estimator data (non-fatal): {err}")
        return ok

    def clear_mempool(self) -> int:
        with self.lock:
            n = len(self.mempool)
            for t in list(self.mempool):
                self.pool_remove(t)
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

    def load_external_block_file(self, path: str) -> int:
        """LoadExternalBlockFile (-loadblock, bootstrap.dat): scan for the network magic, read
        each `magic | u32 size | block` record, and process blocks whose parent is known; blocks
        that arrive before their parent wait until it is connected. Returns blocks accepted."""
        magic = bytes(self.params.message_start)
        act = self.params.kawpow_activation_time
        with open(path, "rb") as f:
            data = f.read()
        waiting: dict[bytes, list] = {}
        n, off = 0, 0

        def process(blk) -> int:
            if not self.process_new_block(blk, check_pow=True).ok:
                return 0
            done, todo = 1, [self.block_hash(blk.header)]
            while todo:
                for child in waiting.pop(todo.pop(), []):
                    if self.process_new_block(child, check_pow=True).ok:
                        done += 1
                        todo.append(self.block_hash(child.header))
            return done

        while True:
            off = data.find(magic, off)
            if off < 0 or off + 8 > len(data):
                break
            size = struct.unpack_from("<I", data, off + 4)[0]
            start = off + 8
            if size < 80 or start + size > len(data):
                off += 1
                continue
            try:
                blk = _core.Block.deserialize(data[start:start + size], act)
            except Exception:
                off += 1
                continue
            off = start + size
            h = self.block_hash(blk.header)
            if self.chain.find(h) is not None and h in self.block_pos:
                continue
            if self.chain.find(blk.header.prev) is None:
                waiting.setdefault(blk.header.prev, []).append(blk)
                continue
            n += process(blk)
        return n

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
        """LoadMempool: every dumped tx goes through AcceptToMemoryPool again (its fee delta
        restored); transactions no longer valid are dropped."""
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
            ok, _, fee = self.accept_to_mempool(tx, test_only=True)
            if ok:
                self.add_to_mempool(tx, fee, float(t), delta)
                n += 1
        return n

    def record_confirmations(self, block, height: int) -> None:
        """removeForBlock -> CBlockPolicyEstimator::processBlock: the block's pool transactions
        are recorded at the number of blocks they waited; blocks at or below the best height the
        estimator has seen (reorgs, side chains) are ignored."""
        self.fee_estimator.process_block(height, [tx.txid() for tx in block.vtx[1:]])
        self._last_rolling_update = self.adjusted_time()  # removeForBlock: the floor starts decaying
        self._block_since_bump = True

    # ------------------------------------------------------------------ ProcessNewBlock
    def check_block_header(self, header) -> ValidationState:
        r = self.chain.check_header(header, True)
        return ValidationState(r.ok, r.reject, r.dos)

    def process_new_block(self, block, check_pow: bool = True) -> ValidationState:
        """Validate + store + activate (ProcessNewBlock). Returns the BIP22-style state of this
        block: invalid if it fails a context-free, contextual, header or connection rule. A
        valid block on a lighter fork is stored (and connected later if its fork wins)."""
        with self.lock:
            h = self.chain.block_hash(block.header)
            existing = self.chain.find(h)
            if existing is not None and (h in self.block_pos or h in self._mem_blocks):
                st = ValidationState.invalid("duplicate")
                self._emit("block_checked", block, st)
                return st
            prev = self.chain.find(block.header.prev)
            ok, reason, dos = _core.check_block(block, self.params, True, self.asset_flags(prev))
            if not ok:
                st = ValidationState.invalid(reason, dos)
                self._emit("block_checked", block, st)
                return st
            if prev is None:
                st = ValidationState.invalid("prev-blk-not-found", 10)
                self._emit("block_checked", block, st)
                return st
            height = prev.height + 1
            ok, reason, dos = _core.contextual_check_block(block, self.params, height)
            if not ok:
                st = ValidationState.invalid(reason, dos)
                self._emit("block_checked", block, st)
                return st
            r = self.chain.accept_header(block.header, self.adjusted_time(), check_pow)
            if not r.ok:
                st = ValidationState.invalid(r.reject, r.dos)
                self._emit("block_checked", block, st)
                return st
            if self.store is not None:
                self.block_pos[h] = self.store.write(block)
                if self.prune_target > 1 and self.block_pos[h].file != getattr(self, "_last_blk_file", -1):
                    self._last_blk_file = self.block_pos[h].file  # a new blk file: look for files to prune
                    self._check_for_pruning = True
                self.index_log.append(block.header.serialize(self.params.kawpow_activation_time), self.block_pos[h],
                                      len(block.vtx), height=height, block_hash=h, time=block.header.time)
            else:
                self.block_pos[h] = None
                self._mem_blocks[h] = block
            self.ntx[h] = len(block.vtx)
            failed = self._activate()
            st = failed.get(h, ValidationState())
            if self.check_block_index_enabled:
                self.check_block_index()
            self._emit("block_checked", block, st)
            return st

    def check_block_index(self) -> None:
        """CheckBlockIndex (-checkblockindex): the active chain links back to genesis one height at
        a time with strictly growing work, its tip is the UTXO set's block, every connected block
        has its data stored, and the best header carries at least the tip's work. Raises
        AssertionError on the first inconsistency."""
        gen = self.chain.genesis()
        tip = self.coins_tip()
        assert tip is not None and self.chain.in_active_chain(tip), "UTXO tip not on the active chain"
        prev = None
        for height in range(0, tip.height + 1):
            idx = self.chain.at_height(height)
            assert idx is not None and idx.height == height, f"active chain hole at {height}"
            if height == 0:
                assert idx.hash == gen.hash, "active chain does not start at genesis"
            else:
                assert idx.prev_hash == prev.hash, f"active chain broken at {height}"
                assert idx.chain_work > prev.chain_work, f"chain work not increasing at {height}"
            assert idx.hash in self.block_pos or idx.hash in self._mem_blocks or height == 0, \
                f"connected block {height} has no data"
            prev = idx
        assert self.chain.tip().chain_work >= tip.chain_work, "best header has less work than the tip"

    # ------------------------------------------------------------------ UTXO set / ActivateBestChain
    def _init_coins(self) -> None:
        """Load the UTXO snapshot and bring it to the best stored chain (ReplayBlocks-lite)."""
        gh = self.chain.genesis().hash
        self.rebuilt = False
        if self.reindex_chainstate and self.coins_path is not None:
            log.log_printf("-reindex-chainstate: rebuilding the chain state from the stored blocks")
        if self.db_format == "leveldb" and self.coins_path is not None:
            # chainstate/ in the reference's layout (CCoinsViewDB): 'C' coins, 'B' best block
            self.coins_db = _core.LevelDB(os.path.dirname(self.coins_path), write_buffer_size=32 << 20)
            self._coins_obf = _core.chaindb_obfuscation_key(self.coins_db, True)
            r = _core.coins_load_ldb(self.coins, self.coins_db, self._coins_obf)
            loaded = r["have_best"] and not r["head_blocks"] and not r["bad"] and not self.reindex_chainstate
            if r["head_blocks"] or r["bad"]:
                log.log_printf(f"chainstate: {'interrupted flush (head blocks)' if r['head_blocks'] else ''}"
                               f"{r['bad']} unreadable coin record(s); rebuilding the UTXO set")
            elif loaded:
                log.log_printf(f"chainstate: {r['coins']} coins loaded")
        else:
            loaded = self.coins_path is not None and not self.reindex_chainstate and \
                self.coins.load_with_journal(self.coins_path, self.coins_log)
        if loaded and self.coins.replayed:
            log.log_printf(f"UTXO journal: {self.coins.replayed} flush record(s) replayed onto the snapshot")
        if loaded and self.coins_db is not None:
            # asset records live in the same store and are flushed in the same batch as the coins
            if not _core.assets_load_ldb(self.assets, self.coins_db, self._coins_obf) or \
                    self.assets.best_block != self.coins.best_block:
                if self._import_reference_assets():
                    pass  # a reference datadir: its assets/ databases describe the chainstate's block
                else:
                    log.log_printf("asset records missing or out of step with the UTXO set; replaying from genesis")
                    loaded = False
            raw = self.coins_db.get(ASSETS_IMPORT_KEY) if loaded else None
            if raw is not None:
                self.assets_import_height = int.from_bytes(_core.chaindb_xor(raw, self._coins_obf)[:4], "little")
        elif loaded:  # the asset state must describe the same block as the UTXO snapshot
            raw = None
            if os.path.exists(self.assets_path):
                with open(self.assets_path, "rb") as f:
                    raw = f.read()
            if raw is None or not self.assets.deserialize(raw) or self.assets.best_block != self.coins.best_block:
                log.log_printf("asset state missing or out of step with the UTXO snapshot; replaying from genesis")
                loaded = False
        if loaded and any(self.index_flags.values()):  # the indexes too (a changed -*index flag replays)
            want = self._new_indexes()
            if self.coins_db is not None:
                # blocks/index records, built with the flags the store recorded ('F')
                at = {(p.file, p.offset): h for h, p in self.block_pos.items() if p is not None}
                ok_load, have_best = _core.indexes_load_ldb(want, self.index_log.db, self.index_log.obf, at)
                if not have_best:
                    # a reference datadir: its ConnectBlock writes the index records with the block,
                    # so they describe at least the chainstate's block
                    want.best_block = self.coins.best_block
                ok = ok_load and all(self._stored_index_flags.get(k) == bool(v) for k, v in self.index_flags.items()) \
                    and self._rewind_indexes(want)
            else:
                raw = None
                if os.path.exists(self.indexes_path):
                    with open(self.indexes_path, "rb") as f:
                        raw = f.read()
                ok = raw is not None and want.deserialize(raw) and \
                    all(getattr(want, k) == bool(v) for k, v in self.index_flags.items()) and self._rewind_indexes(want)
            if ok:
                self.indexes = want
            else:
                log.log_printf("chain indexes missing or built with other flags; replaying from genesis")
                loaded = False
        if (not loaded or self.chain.find(self.coins.best_block) is None) and self.have_pruned:
            # replaying from genesis needs every block, and the pruned ones are gone
            raise SystemExit("Unable to rebuild the chain state: block files were pruned. "
                             "You will need to rebuild the database using -reindex.")
        if not loaded or self.chain.find(self.coins.best_block) is None:
            if loaded:
                log.log_printf("UTXO snapshot's best block is unknown; rebuilding the UTXO set from genesis")
            self.coins = _core.CoinsView()
            self.coins.best_block = gh  # the genesis coinbase is unspendable: never added
            self.assets = _core.AssetsState()
            self.indexes = self._new_indexes()
            self.indexes.best_block = gh
            self.rebuilt = self.coins_path is not None  # start-up replayed the chain from genesis
            if self.coins_db is not None:
                # drop the stale set: every coin record, then the fresh (empty) state's 'B'
                stale = [(k, None) for k, _ in self.coins_db.items(b"C", b"D")]
                stale += [(k, None) for k, _ in self.coins_db.items(b"\x01", b"\x02")]  # asset records
                # a replay rebuilds every block's asset undo: no import height survives it
                self.coins_db.write(stale + [(b"H", None), (ASSETS_IMPORT_KEY, None)])
                self.assets.best_block = gh
                _core.coins_flush_ldb(self.coins, self.coins_db, self._coins_obf, True, self.assets)
                _core.indexes_purge_ldb(self.index_log.db)  # the indexes are rebuilt by the replay
            elif self.coins_path is not None and (os.path.exists(self.coins_path) or os.path.exists(self.coins_log)):
                self.coins.compact(self.coins_path, self.coins_log)  # a fresh snapshot restarts the journal
        with self.lock:
            self._activate()

    def _import_reference_assets(self) -> bool:
        """A reference datadir's asset state: CAssetsDB (`assets/`) and CRestrictedDB
        (`assets/restricted`), which the reference flushes together with its chainstate
        (src/validation.cpp FlushStateToDisk), read into this engine's asset records
        (csrc/store/chaindb.cpp assets_import_reference) and written to chainstate/ in the same
        batch as 'B', so the node opens without replaying the chain. Blocks the reference
        connected have no asset undo records of this engine: the import height is kept, and a
        reorg that would disconnect one of them with asset activity asks for -reindex-chainstate
        (as the reference does for a missing undo, src/validation.cpp DisconnectBlock).

        Runs at most once per datadir: with an import marker or any engine asset record present it
        returns False (the caller replays). The reference flushes its coins before its asset
        databases (src/validation.cpp:10693-10703), so an interrupted reference flush can leave
        assets/ one flush behind its chainstate; nothing in assets/ records a block to check that
        against, which is why the import is confined to the first open."""
        if not self.datadir:
            return False
        # only the first open of a reference datadir imports: once this engine has written asset
        # records (or imported once), assets/ is stale — the engine advances the chain without it —
        # and a later load failure or mismatch must replay from genesis, never re-import
        if self.coins_db.get(ASSETS_IMPORT_KEY) is not None or self.coins_db.get(b"\x02assets.best") is not None or \
                next(iter(self.coins_db.items(b"\x01", b"\x02")), None) is not None:
            return False
        adir = os.path.join(self.datadir, "assets")
        if not os.path.exists(os.path.join(adir, "CURRENT")):
            return False
        tip = self.chain.find(self.coins.best_block)
        if tip is None:
            return False
        rdir = os.path.join(adir, "restricted")
        adb = _core.LevelDB(adir, create_if_missing=False)
        rdb = _core.LevelDB(rdir, create_if_missing=False) if os.path.exists(os.path.join(rdir, "CURRENT")) else None
        try:
            st = _core.AssetsState()
            r = _core.assets_import_reference_ldb(st, adb, rdb)
        finally:
            adb.close()
            if rdb is not None:
                rdb.close()
        if r["bad"]:
            log.log_printf(f"assets/: {r['bad']} unreadable record(s); replaying the asset state instead")
            return False
        st.best_block = self.coins.best_block
        st.mark_all_dirty()
        self.assets = st
        self.assets_import_height = int(tip.height)
        self.coins_db.write([(ASSETS_IMPORT_KEY, _core.chaindb_xor(int(tip.height).to_bytes(4, "little"),
                                                                   self._coins_obf))])
        _core.coins_flush_ldb(self.coins, self.coins_db, self._coins_obf, True, self.assets)
        log.log_printf(f"assets/: imported {r['assets']} assets, {r['balances']} balances, {r['tags']} tags, "
                       f"{r['restrictions']} restrictions, {r['global_restrictions']} global restrictions and "
                       f"{r['verifiers']} verifiers at height {tip.height}")
        return True

    @staticmethod
    def _block_has_asset_ops(blk) -> bool:
        for tx in blk.vtx:
            for o in tx.vout:
                if _core.parse_asset_script(o.script_pubkey) is not None or \
                        _core.parse_null_asset_script(o.script_pubkey) is not None:
                    return True
        return False

    def _rewind_indexes(self, ix) -> bool:
        """Bring loaded indexes to the UTXO set's block. A flush writes the index records before the
        coins, so a crash between the two leaves the indexes ahead of the chainstate by the blocks of
        one flush interval; their index changes are undone here from the stored blocks and undo data
        (ChainIndexes.disconnect), and the start-up replay then connects those blocks — coins and
        index together — exactly once. (The reference writes index records with each block and
        reconnects idempotently; rewinding keeps the in-memory delta lists free of duplicates.)
        False when the index is not on the chainstate's chain or a block needed is missing."""
        have, want = self.coins.best_block, ix.best_block
        if want == have:
            return True
        a, b = self.chain.find(want), self.chain.find(have)
        if a is None or b is None or a.height <= b.height:
            return False
        path, cur = [], a
        while cur is not None and cur.height > b.height:
            path.append(cur)
            cur = self.chain.find(cur.prev_hash)
        if cur is None or cur.hash != have:
            return False
        for x in path:  # newest first
            blk = self.get_block(x.hash)
            undo = self.undo.read(x.hash, x.prev_hash)
            if blk is None or undo is None:
                return False
            ix.disconnect(blk, x.height, x.hash, undo)
        log.log_printf(f"chain indexes were {len(path)} block(s) ahead of the UTXO set (interrupted flush); "
                       f"rewound to {_core.u256_hex(have)}")
        return ix.best_block == have

    def coins_tip(self):
        return self.chain.find(self.coins.best_block)

    def asset_flags(self, prev):
        """Asset deployments in force for the block after `prev` (AreAssetsDeployed,
        AreMessagesDeployed / AreRestrictedAssetsDeployed, AreEnforcedValuesDeployed,
        AreCoinbaseCheckAssetsDeployed: src/validation.cpp:13441-13510)."""
        if prev is None:
            return _core.AssetFlags()
        states = {d.name: self.versionbits.state_for(prev, d) for d in self.versionbits.deployments}
        return _core.AssetFlags(states.get("assets") == "active", states.get("messaging_restricted") == "active",
                                states.get("enforce_value") in ("active", "locked_in"), states.get("coinbase") == "active")

    def invalidate_block(self, h: bytes) -> None:
        """InvalidateBlock: mark the block (and its descendants) invalid and move the UTXO set to
        the best remaining chain; the disconnected transactions go back to the mempool."""
        with self.lock:
            self.chain.invalidate(h)
            self._activate()

    def reconsider_block(self, h: bytes) -> None:
        """ReconsiderBlock: clear the invalid flags and re-activate the best chain."""
        with self.lock:
            self.chain.reconsider(h)
            self._activate()

    def _fork_point(self, a, b):
        while a.height > b.height:
            a = self.chain.find(a.prev_hash)
        while b.height > a.height:
            b = self.chain.find(b.prev_hash)
        while a.hash != b.hash:
            a, b = self.chain.find(a.prev_hash), self.chain.find(b.prev_hash)
        return a

    def _activate(self) -> dict[bytes, ValidationState]:
        """ActivateBestChain: move the UTXO set from its tip to the header chain's best tip,
        disconnecting to the fork point and connecting every block whose data is stored. A block
        that fails is marked invalid in the header chain (which re-selects its tip) and the walk
        restarts. Returns the failed blocks' states."""
        failed: dict[bytes, ValidationState] = {}
        old_tip = self.coins_tip()
        disconnected = []
        connected = []
        while True:
            target = self.chain.tip()
            cur = self.coins_tip()
            if cur.hash == target.hash:
                break
            fork = self._fork_point(cur, target)
            while cur.hash != fork.hash:
                blk = self.get_block(cur.hash)
                undo = self.undo.read(cur.hash, cur.prev_hash)
                if blk is None or undo is None:
                    raise RuntimeError(f"cannot disconnect {_core.u256_hex(cur.hash)}: block or undo data missing")
                aundo = self.asset_undo.read(cur.hash, cur.prev_hash)
                if aundo is None and cur.height <= self.assets_import_height and self._block_has_asset_ops(blk):
                    # connected by the reference node (assets/ imported): no undo record of this engine
                    raise RuntimeError(f"cannot disconnect {_core.u256_hex(cur.hash)}: its asset undo data is in "
                                       "the reference's format; restart with -reindex-chainstate")
                aundo = aundo or b""
                if not _core.disconnect_block(blk, undo, self.coins, self.assets, aundo):
                    log.log_printf(f"disconnect of {_core.u256_hex(cur.hash)} found an inconsistent UTXO set")
                self.indexes.disconnect(blk, cur.height, cur.hash, undo)
                self.coins.best_block = cur.prev_hash
                self._emit("disconnect_tip", blk, cur, undo)
                disconnected.append(blk)
                cur = self.chain.find(cur.prev_hash)
            path, x = [], target
            while x.hash != fork.hash:
                path.append(x)
                x = self.chain.find(x.prev_hash)
            restart = False
            for idx in reversed(path):
                blk = self.get_block(idx.hash)
                if blk is None:
                    break  # data not here yet (headers-first): stop at the last complete block
                st = self._connect_one(blk, idx)
                if not st.ok:
                    failed[idx.hash] = st
                    self.chain.invalidate(idx.hash)
                    restart = True
                    break
                connected.append((blk, idx))
            if not restart:
                break
        if disconnected or connected:
            self._update_mempool(disconnected, [b for b, _ in connected])
            for blk, idx in connected:
                self._emit("block_connected", blk, idx)
            new_tip = self.coins_tip()
            if new_tip.hash != old_tip.hash:
                self._emit("updated_block_tip", new_tip, old_tip, False)
                self.cv_tip.notify_all()
                log.log_print("validation", f"new tip {_core.u256_hex(new_tip.hash)} height {new_tip.height}")
        return failed

    def _use_gpu_for(self, block) -> bool:
        if self.gpu_signatures == "off":
            return False
        n_inputs = sum(len(tx.vin) for tx in block.vtx[1:])
        if n_inputs < (1 if self.gpu_signatures == "on" else GPU_SIG_BATCH_MIN):
            return False
        try:
            import torch

            return torch.cuda.is_available()
        except ImportError:  # pragma: no cover
            return False

    def _connect_one(self, block, idx) -> ValidationState:
        """ConnectTip: connect `block` at `idx`, then the coinbase / community-fund rules on the
        block's real fees; on any failure the UTXO set is left as it was."""
        height = idx.height
        prev = self.chain.find(idx.prev_hash)
        mtp_prev = prev.median_time_past()

        def mtp_at(h: int) -> int:
            return self.chain.at_height(h).median_time_past()

        flags = _core.BLOCK_SCRIPT_VERIFY_FLAGS
        check_scripts = not self._assumed_valid(idx)
        if not check_scripts:
            self.scripts_skipped += 1
        gpu = check_scripts and self._use_gpu_for(block)
        par = self.script_threads
        aflags = self.asset_flags(prev)

        def connect(defer: bool):
            return _core.connect_block(block, height, self.coins, check_scripts, defer, mtp_at, mtp_prev, flags, par,
                                       self.assets, aflags, idx.hash)

        res, undo = connect(gpu)
        if gpu and not res.ok and "script-verify" in res.reject:
            # a deferred (assume-valid) signature can flip a script that depends on a signature
            # failing: the host run decides
            res, undo = connect(False)
        if not res.ok:
            return ValidationState.invalid(res.reject, res.dos)
        aundo = res.asset_undo
        if gpu and res.num_sigs:
            from ..ops import secp

            verdicts = secp.verify_batch(res.sig_items())
            self.sig_stats["gpu_batches"] += 1
            self.sig_stats["gpu_sigs"] += len(verdicts)
            for t, i in sorted({res.sig_at[k] for k, v in enumerate(verdicts) if not v}):
                value, spk, _, _ = _core.block_undo_coin(undo, t, i)
                self.sig_stats["host_rechecks"] += 1
                ok, err = _core.verify_input_host(block, t, i, value, spk, flags)
                if not ok:
                    _core.disconnect_block(block, undo, self.coins, self.assets, aundo)
                    return ValidationState.invalid(f"mandatory-script-verify-flag-failed ({err})", 100)
        ok, reason, dos = _core.check_coinbase_rewards(block, self.params, height, res.fees, True)
        if not ok:
            _core.disconnect_block(block, undo, self.coins, self.assets, aundo)
            return ValidationState.invalid(reason, dos)
        bpos = self.block_pos.get(idx.hash)
        if self.db_format == "leveldb" and bpos is not None:
            u = self.undo.pos.get(idx.hash)
            if u is None or u[0] != bpos.file:  # written once, beside the block (WriteUndoDataForBlock)
                u = self.undo.write(idx.hash, idx.prev_hash, undo, file=bpos.file)
            self.index_log.set_undo(idx.hash, u[0], u[1], u[2])
        else:
            self.undo.write(idx.hash, idx.prev_hash, undo)
        if bpos is not None:
            self.indexes.connect(block, height, idx.hash, undo, bpos.file, bpos.offset)
        else:
            self.indexes.connect(block, height, idx.hash, undo)
        if aundo:  # beside the block's file too, so pruning a blk file drops its asset undo with it
            self.asset_undo.write(idx.hash, idx.prev_hash, aundo, file=bpos.file if bpos is not None else None)
        self.coins.best_block = idx.hash
        self.record_confirmations(block, height)
        self._emit("connect_tip", block, idx, undo)
        self._since_flush += 1
        if self._since_flush >= self.flush_interval or self._check_for_pruning or \
                self.coins.dirty * COIN_CACHE_ENTRY_BYTES > self.coins_cache_bytes:
            self.flush()
        return ValidationState()

    def flush(self) -> None:
        """FlushStateToDisk: write the UTXO snapshot (atomically) if anything changed."""
        if self.coins_path is None or self._since_flush == 0:
            return
        os.makedirs(os.path.dirname(self.coins_path), exist_ok=True)
        self.assets.best_block = self.coins.best_block
        if self.coins_db is None:
            # assets.dat first: a crash between the two leaves an asset state that does not match
            # the UTXO snapshot, which start-up detects (and replays) instead of mixing two states
            tmp = self.assets_path + ".new"
            with open(tmp, "wb") as f:
                f.write(self.assets.serialize())
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, self.assets_path)
        if self.coins_db is None:
            self._maybe_crash()
        if any(self.index_flags.values()) and self.coins_db is not None:
            # the index changes since the last flush, as blocks/index records (made durable by the
            # synced block-tree write below)
            _core.indexes_flush_ldb(self.indexes, self.index_log.db, self.index_log.obf, False)
        elif any(self.index_flags.values()):
            tmp = self.indexes_path + ".new"
            with open(tmp, "wb") as f:
                f.write(self.indexes.serialize())
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, self.indexes_path)
        if self.coins_db is not None:
            # block index records first (their undo positions must be durable before the coins
            # that depend on them), then the UTXO and asset change sets with 'B' in one synced batch
            self.index_log.sync()
            self._maybe_crash()  # blocks and their index durable, the UTXO set still at the last flush
            _core.coins_flush_ldb(self.coins, self.coins_db, self._coins_obf, True, self.assets)
        elif not os.path.exists(self.coins_path):  # first flush of this datadir: start from a snapshot
            self.coins.compact(self.coins_path, self.coins_log)
        else:
            self.coins.append_journal(self.coins_log)  # O(outputs changed since the last flush)
            if os.path.getsize(self.coins_log) > max(self.journal_compact_bytes, os.path.getsize(self.coins_path)):
                self.coins.compact(self.coins_path, self.coins_log)
        self._since_flush = 0
        if self._check_for_pruning:
            # FlushStateToDisk -> FindFilesToPrune: only after the UTXO set and the block index
            # are durable, so no state still needs what the deleted files held
            self._check_for_pruning = False
            self.prune_block_files(self.files_to_prune())

    # ------------------------------------------------------------------ pruning
    @property
    def prune_mode(self) -> bool:
        return self.prune_target > 0

    @property
    def have_pruned(self) -> bool:
        return bool(self.index_log is not None and hasattr(self.index_log, "flag")
                    and self.index_log.flag("prunedblockfiles"))

    def _blk_file_bytes(self, fi: int) -> int:
        n = 0
        for path in (self.store.path(fi), self.undo._path(fi), self.asset_undo._path(fi)):
            try:
                n += os.path.getsize(path)
            except OSError:
                pass
        return n

    def files_to_prune(self, manual_height: int | None = None) -> list[int]:
        """FindFilesToPrune / FindFilesToPruneManual (src/validation.cpp:12255-12343): blk files
        (never the one being written) whose highest block is at least MIN_BLOCKS_TO_KEEP below the
        tip; automatic pruning takes them oldest first until the files, plus a chunk of headroom,
        fit under the -prune target, manual pruning takes every one at or below `manual_height`."""
        if not self.prune_mode or self.store is None or not hasattr(self.index_log, "files"):
            return []
        tip = self.chain.height()
        if tip <= self.prune_after_height:
            return []
        last_ok = tip - MIN_BLOCKS_TO_KEEP
        if manual_height is not None:
            last_ok = min(last_ok, manual_height)
        current = self.store.current_file()
        files = sorted(f for f, info in self.index_log.files.items() if f < current and info[0] > 0)
        if manual_height is not None:
            return [f for f in files if self.index_log.files[f][4] <= last_ok]
        if self.prune_target <= 1:
            return []
        usage = sum(self._blk_file_bytes(f) for f in range(current + 1))
        buffer = BLOCKFILE_CHUNK_SIZE + UNDOFILE_CHUNK_SIZE
        out = []
        for f in files:
            if usage + buffer < self.prune_target:
                break
            if self.index_log.files[f][4] > last_ok:
                continue
            out.append(f)
            usage -= self._blk_file_bytes(f)
        return out

    def prune_block_files(self, files: list[int]) -> int:
        """PruneOneBlockFile + UnlinkPrunedFiles: forget the files' blocks and undo data, mark
        the store as pruned ('F' prunedblockfiles) and delete blk/rev files. Returns the count."""
        if not files:
            return 0
        with self.lock:
            self.flush()
            if not self.have_pruned:
                self.index_log.set_flag("prunedblockfiles", True)
            for f in files:
                for h in self.index_log.prune_file(f):
                    self.block_pos.pop(h, None)
                self.index_log.sync()
                self.undo.drop_file(f)
                self.asset_undo.drop_file(f)
                try:
                    os.remove(self.store.path(f))
                except OSError:
                    pass
                log.log_print("prune", f"Prune: deleted blk/rev ({f:05d})")
        return len(files)

    def prune_height(self) -> int:
        """getblockchaininfo.pruneheight: the lowest height from which every active-chain block
        down from the tip still has its data."""
        idx = self.chain.tip()
        while idx.height > 0:
            prev = self.chain.find(idx.prev_hash)
            if prev is None or prev.hash not in self.block_pos:
                break
            idx = prev
        return idx.height

    def _maybe_crash(self) -> None:
        if self.db_crash_ratio and random.randrange(self.db_crash_ratio) == 0:
            # -dbcrashratio (CCoinsViewDB::BatchWrite, src/txdb.cpp:96): die between the two halves
            # of the flush; start-up must notice the mismatch and replay (feature_dbcrash.py)
            log.log_printf("Simulating a crash. Goodbye.")
            os._exit(0)

    def chainstate_disk_size(self) -> int:
        """gettxoutsetinfo.disk_size (CCoinsViewDB::EstimateSize): bytes of the chainstate store."""
        if self.coins_db is not None:
            # the tables, plus the write-ahead log that holds what has not reached a table yet
            d = os.path.dirname(self.coins_path)
            return int(self.coins_db.disk_bytes) + sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d)
                                                        if f.endswith(".log") and f != "LOG")
        return sum(os.path.getsize(p) for p in (self.coins_path, self.coins_log, self.assets_path)
                   if p is not None and os.path.exists(p))

    def _update_mempool(self, disconnected, connected) -> None:
        """UpdateMempoolForReorg + removeForBlock: drop what the new blocks confirmed or
        conflict with, return the disconnected blocks' transactions to the pool where they are
        still valid, and evict anything whose inputs are gone."""
        confirmed = {tx.txid() for blk in connected for tx in blk.vtx[1:]}
        spent = {(i.prevout.hash, i.prevout.n) for blk in connected for tx in blk.vtx[1:] for i in tx.vin}
        for txid in list(self.mempool):
            e = self.mempool[txid]
            if txid in confirmed or any((i.prevout.hash, i.prevout.n) in spent for i in e.tx.vin):
                self.pool_remove(txid, txid in confirmed)
        for blk in reversed(disconnected):
            for tx in blk.vtx[1:]:
                self.accept_to_mempool(tx)
        # evict transactions whose inputs are neither unspent outputs nor pool outputs
        changed = True
        while changed:
            changed = False
            for txid in list(self.mempool):
                e = self.mempool[txid]
                for i in e.tx.vin:
                    if self.coins.get(i.prevout.hash, i.prevout.n) is None and i.prevout.hash not in self.mempool:
                        self.pool_remove(txid)
                        changed = True
                        break
        self.transactions_updated += 1

    # ------------------------------------------------------------------ AcceptToMemoryPool
    def _spent_coin(self, prevout):
        """(value, scriptPubKey, height, coinbase) of an unspent output, from the UTXO set or a
        pool transaction (height = next block)."""
        c = self.coins.get(prevout.hash, prevout.n)
        if c is not None:
            return c
        e = self.mempool.get(prevout.hash)
        if e is not None and prevout.n < len(e.tx.vout):
            o = e.tx.vout[prevout.n]
            return (o.value, o.script_pubkey, self.coins_tip().height + 1, False)
        return None

    def mempool_sigop_cost(self, txid: bytes) -> int:
        """GetTransactionSigOpCost of a pool transaction (cached on its entry; computed from the
        spent outputs when the entry predates it, e.g. one loaded from mempool.dat)."""
        with self.lock:
            e = self.mempool[txid]
            if e.sigop_cost < 0:
                spent = [self._spent_coin(i.prevout) for i in e.tx.vin]
                if any(c is None for c in spent):  # inputs gone: count what needs no spent outputs
                    return _core.tx_legacy_sigops(e.tx.serialize(True)) * 4
                e.sigop_cost = _core.tx_sigop_cost(e.tx.serialize(True), [c[1] for c in spent],
                                                   _core.STANDARD_SCRIPT_VERIFY_FLAGS)
            return e.sigop_cost

    def accept_to_mempool(self, tx, test_only: bool = False, max_fee: int | None = None) -> tuple[bool, str, int]:
        """AcceptToMemoryPoolWorker (src/validation.cpp): context-free checks, standardness,
        inputs present (UTXO set or pool), no pool conflict, coinbase maturity, fees and the
        min relay fee, then every input script under the standard flags. Returns (accepted,
        reject reason, fee)."""
        with self.lock:
            txid = tx.txid()
            if txid in self.mempool:
                return False, "txn-already-in-mempool", 0
            raw = tx.serialize(True)
            aflags = self.asset_flags(self.coins_tip())
            why = _core.check_transaction(raw, self.params, aflags, False, True)
            if why:
                return False, why, 0
            if tx.is_coinbase():
                return False, "coinbase", 0
            weight = len(tx.serialize(False)) * 3 + len(raw)
            if self.require_standard:  # IsStandardTx (fRequireStandard: mainnet, or !-acceptnonstdtxn)
                if tx.version < 1 or tx.version > 2:
                    return False, "version", 0
                if weight >= MAX_STANDARD_TX_WEIGHT:
                    return False, "tx-size", 0
                for i in tx.vin:
                    if len(i.script_sig) > MAX_STANDARD_SCRIPTSIG_SIZE:
                        return False, "scriptsig-size", 0
                    if not _core.script_is_push_only(i.script_sig):
                        return False, "scriptsig-not-pushonly", 0
                why = policy.standard_outputs_reason(tx, permit_bare_multisig=self.permit_bare_multisig,
                                                     datacarrier=self.datacarrier,
                                                     datacarrier_size=self.datacarrier_size,
                                                     dust_fee=self.dust_relay_fee)
                if why:
                    return False, why, 0
            pool_spent = {(i.prevout.hash, i.prevout.n): t for t, e in self.mempool.items() for i in e.tx.vin}
            tip = self.coins_tip()
            next_height = tip.height + 1
            # CheckFinalTx for the next block (IsFinalTx with the tip's median time past)
            if tx.lock_time != 0 and any(i.sequence != 0xffffffff for i in tx.vin):
                limit = next_height if tx.lock_time < 500_000_000 else tip.median_time_past()
                if tx.lock_time >= limit:
                    return False, "non-final", 0
            in_sum, coins = 0, []
            conflicts = {pool_spent[(i.prevout.hash, i.prevout.n)] for i in tx.vin
                         if (i.prevout.hash, i.prevout.n) in pool_spent}
            if conflicts and (not self.enable_replacement
                              or not all(policy.signals_rbf(self.mempool[t].tx) for t in conflicts)):
                return False, "txn-mempool-conflict", 0
            for i in tx.vin:
                c = self._spent_coin(i.prevout)
                if c is None:
                    return False, "missing-inputs", 0
                value, spk, h, coinbase = c
                if coinbase and next_height - h < _core.COINBASE_MATURITY:
                    return False, "bad-txns-premature-spend-of-coinbase", 0
                in_sum += value
                coins.append((value, spk))
            fee = in_sum - tx.value_out()
            if fee < 0:
                return False, "bad-txns-in-belowout", 0
            # GetTransactionSigOpCost with the spent outputs (P2SH redeem scripts, witness programs)
            sigop_cost = _core.tx_sigop_cost(raw, [spk for _, spk in coins], _core.STANDARD_SCRIPT_VERIFY_FLAGS)
            if sigop_cost > MAX_STANDARD_TX_SIGOPS_COST:
                return False, "bad-txns-too-many-sigops", fee
            why = self._check_tx_assets(tx, raw, coins, aflags)
            if why:
                return False, why, 0
            vsize = (max(weight, sigop_cost * self.bytes_per_sigop) + 3) // 4  # GetVirtualTransactionSize
            pool_floor = self.mempool_min_fee() * vsize // 1000
            if pool_floor > 0 and fee < pool_floor:
                return False, f"mempool min fee not met, {fee} < {pool_floor}", fee
            if fee < self.min_relay_fee * vsize // 1000:
                return False, "min relay fee not met", fee
            replaced = set()
            if conflicts:
                why, replaced = self._check_replacement(tx, fee, vsize, conflicts)
                if why:
                    return False, why, fee
            if max_fee is not None and fee > max_fee:
                return False, "absurdly-high-fee", fee
            why = self._check_package_limits(tx, vsize, conflicts | replaced)
            if why:
                return False, why, fee
            for k, (value, spk) in enumerate(coins):
                vin = tx.vin[k]
                # sigcache=1: signatures that verify are remembered, so the block that confirms this
                # transaction skips them (CSignatureCache, src/script/sigcache.cpp:76-86)
                ok, err = _core.verify_script(vin.script_sig, spk, list(vin.witness), _core.STANDARD_SCRIPT_VERIFY_FLAGS,
                                              raw, k, value, 1)
                if not ok:
                    ok2, _ = _core.verify_script(vin.script_sig, spk, list(vin.witness),
                                                 _core.BLOCK_SCRIPT_VERIFY_FLAGS, raw, k, value)
                    kind = "non-mandatory-script-verify-flag" if ok2 else "mandatory-script-verify-flag-failed"
                    return False, f"{kind} ({err})", fee
            if not test_only:
                # BIP125: the replaced transactions and their descendants leave (kept aside for
                # compact-block reconstruction: vExtraTxnForCompact)
                self.last_replaced = [self.mempool[t].tx for t in replaced if t in self.mempool]
                for t in replaced:
                    self.pool_remove(t)
                self.add_to_mempool(tx, fee, replacement=bool(replaced), sigop_cost=sigop_cost)
                self.expire_mempool()  # LimitMempoolSize -> Expire, TrimToSize
                self.trim_mempool()
                if txid not in self.mempool:
                    return False, "mempool full", fee
            return True, "", fee

    def _check_package_limits(self, tx, vsize: int, leaving: set) -> str:
        """CalculateMemPoolAncestors with -limitancestorcount / -limitancestorsize and, for each
        ancestor, -limitdescendantcount / -limitdescendantsize (transactions being replaced do not
        count). Returns "" or "too-long-mempool-chain"."""
        parents = {i.prevout.hash for i in tx.vin if i.prevout.hash in self.mempool and i.prevout.hash not in leaving}
        if not parents:
            return ""
        anc = set(parents)
        for p in parents:
            anc |= self.mempool_ancestors(p)
        anc -= leaving
        n_max, size_max = self.ancestor_limits
        if len(anc) + 1 > n_max or sum(self.mempool[a].vsize() for a in anc) + vsize > size_max:
            return "too-long-mempool-chain"
        d_max, dsize_max = self.descendant_limits
        for a in anc:
            desc = self.mempool_descendants(a) - leaving
            if len(desc) + 2 > d_max or (self.mempool[a].vsize() + sum(self.mempool[d].vsize() for d in desc)
                                         + vsize) > dsize_max:
                return "too-long-mempool-chain"
        return ""

    def expire_mempool(self, now: float | None = None) -> int:
        """CTxMemPool::Expire: entries older than -mempoolexpiry leave with their descendants."""
        cutoff = (self.adjusted_time() if now is None else now) - self.mempool_expiry
        with self.lock:
            old = [t for t, e in self.mempool.items() if e.time < cutoff]
            gone = set(old)
            for t in old:
                gone |= self.mempool_descendants(t)
            for t in gone:
                self.pool_remove(t)
            if gone:
                self.transactions_updated += 1
        return len(gone)

    def _check_replacement(self, tx, fee: int, vsize: int, conflicts: set) -> tuple[str, set]:
        """The BIP125 rules of AcceptToMemoryPoolWorker (src/validation.cpp, -mempoolreplacement):
        a higher feerate than every direct conflict, at most 100 evicted transactions (conflicts
        and their descendants), no spend of an evicted transaction, no new unconfirmed inputs, a
        fee covering the evicted fees plus the incremental relay fee for this transaction."""
        evict = set(conflicts)
        frontier = list(conflicts)
        while frontier:
            t = frontier.pop()
            for c, e in self.mempool.items():
                if c not in evict and any(i.prevout.hash == t for i in e.tx.vin):
                    evict.add(c)
                    frontier.append(c)
            if len(evict) > policy.MAX_BIP125_REPLACEMENTS:
                return "too many potential replacements", set()
        for t in conflicts:
            e = self.mempool[t]
            if fee * max(1, e.size) <= e.fee * vsize:  # new feerate must beat each direct conflict's
                return "insufficient fee", set()
        if any(i.prevout.hash in evict for i in tx.vin):
            return "bad-txns-spends-conflicting-tx", set()
        old_parents = {i.prevout.hash for t in conflicts for i in self.mempool[t].tx.vin}
        for i in tx.vin:
            if i.prevout.hash in self.mempool and i.prevout.hash not in old_parents:
                return "replacement-adds-unconfirmed", set()
        evicted_fees = sum(self.mempool[t].fee for t in evict)
        if fee < evicted_fees:
            return "insufficient fee", set()
        if fee - evicted_fees < self.incremental_relay_fee * vsize // 1000:
            return "insufficient fee", set()
        return "", evict

    def _check_tx_assets(self, tx, raw: bytes, coins, aflags) -> str:
        """The asset part of ATMP: no asset outputs before the deployment, CheckTxAssets against the
        current asset state, names already being created in the pool (mapAssetToHash) and one
        reissue per asset in the pool (mapReissuedAssets)."""
        kinds = [_core.parse_asset_script(o.script_pubkey) for o in tx.vout]
        nulls = [_core.parse_null_asset_script(o.script_pubkey) for o in tx.vout]
        if not aflags.assets:
            if any(kinds):
                return "bad-txns-is-asset-and-asset-not-active"
            if any(nulls):
                return "bad-tx-null-asset-data-before-restricted-assets-activated"
            return ""
        pending, reissued = set(), set()
        for e in self.mempool.values():
            for o in e.tx.vout:
                a = _core.parse_asset_script(o.script_pubkey)
                if a is not None and a["type"] == "new_asset":
                    pending.add(a["name"])
                elif a is not None and a["type"] == "reissue_asset":
                    reissued.add(a["name"])
        for a in kinds:
            if a is not None and a["type"] == "reissue_asset" and a["name"] in reissued:
                return "bad-tx-reissue-chaining-not-allowed"
        return _core.check_tx_assets(raw, coins, self.assets, aflags, pending)

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

