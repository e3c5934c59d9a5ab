"""Asset ownership snapshots and reward distribution (SURVEY S10 rewards, A5 "rewards" RPC family).

Parity (behaviour):
* CSnapshotRequestDB (src/assets/snapshotrequestdb.cpp): scheduled (asset, height) snapshot
  requests; CAssetSnapshotDB::AddAssetOwnershipSnapshot (src/assets/assetsnapshotdb.cpp:38) takes
  the owner list of the asset when the block at that height is connected (ConnectTip,
  src/validation.cpp:11058-11078).
* CRewardSnapshot (src/assets/rewards.h:83): its hash is the double-SHA256 of the serialized
  (ownership asset, distribution asset, exception addresses, amount, height) without the status,
  so getdistributestatus finds a distribution from the same five arguments.
* GenerateDistributionList / DistributeRewardSnapshot / BuildTransaction (src/assets/rewards.cpp):
  exception and burn addresses are dropped, every other owner gets amount * owned / total, cut to
  the distribution asset's units, in batches of MAX_PAYMENTS_PER_TRANSACTION outputs; a batch
  whose transaction is already recorded is skipped while it is in the pool or confirmed; failures
  set the status codes of the reference (LOW_FUNDS 3, NOT_ENOUGH_FEE 4, LOW_REWARDS 5,
  FAILED_CREATE_TRANSACTION 8, FAILED_COMMIT_TRANSACTION 9) and every later block retries
  (CheckRewardDistributions). One addition: once every batch is confirmed the status becomes
  COMPLETE (2), a code the reference defines but never sets.

The reference's per-owner share is computed in long double; here it is exact integer arithmetic
(floor(owned * amount / total)), which can differ by one unit of the distribution asset only where
the long-double product rounds below an exact integer (parity unpinned at that edge).
State lives in `<datadir>/rewards.json` (atomic replace) instead of three LevelDB databases.
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import threading

from .. import core
from ..chain.state import ValidationInterface
from ..utils import log
from .wallet import WalletError

_core = core()
COIN = 100_000_000
MAX_PAYMENTS_PER_TRANSACTION = 1000
MINIMUM_REWARDS_PAYOUT_HEIGHT = 60

REWARD_ERROR, PROCESSING, COMPLETE, LOW_FUNDS, NOT_ENOUGH_FEE, LOW_REWARDS, STUCK_TX, NETWORK_ERROR, \
    FAILED_CREATE_TRANSACTION, FAILED_COMMIT_TRANSACTION = range(10)


def _ser_str(s: str) -> bytes:
    b = s.encode()
    n = len(b)
    if n < 253:
        return bytes([n]) + b
    if n <= 0xFFFF:
        return b"\xfd" + struct.pack("<H", n) + b
    return b"\xfe" + struct.pack("<I", n) + b


class RewardSnapshot:
    __slots__ = ("owner_asset", "dist_asset", "exceptions", "amount", "height", "status")

    def __init__(self, owner_asset: str, dist_asset: str, exceptions: str, amount: int, height: int,
                 status: int = PROCESSING):
        self.owner_asset, self.dist_asset, self.exceptions = owner_asset, dist_asset, exceptions
        self.amount, self.height, self.status = amount, height, status

    def hash(self) -> bytes:
        """SerializeHash(*this, SER_GETHASH): the status is not part of the hash."""
        raw = (_ser_str(self.owner_asset) + _ser_str(self.dist_asset) + _ser_str(self.exceptions)
               + struct.pack("<qI", self.amount, self.height))
        return hashlib.sha256(hashlib.sha256(raw).digest()).digest()

    def to_json(self) -> dict:
        return {k: getattr(self, k) for k in self.__slots__}


class Rewards(ValidationInterface):
    def __init__(self, state, wallet, asset_wallet_fn, path: str | None, min_reward_height: int =
                 MINIMUM_REWARDS_PAYOUT_HEIGHT):
        self.state = state
        self.wallet = wallet
        self._asset_wallet = asset_wallet_fn  # lazily built AssetWallet (shared with the asset RPCs)
        self.path = path
        self.min_reward_height = min_reward_height
        self.lock = threading.RLock()
        self.requests: set[tuple[str, int]] = set()
        self.snapshots: dict[tuple[str, int], list[tuple[str, int]]] = {}
        self.distributions: dict[bytes, RewardSnapshot] = {}
        self.batch_txids: dict[tuple[bytes, int], bytes] = {}
        if path and os.path.exists(path):
            self._load()

    # ------------------------------------------------------------------ persistence
    def _load(self) -> None:
        with open(self.path) as f:
            d = json.load(f)
        self.requests = {(n, h) for n, h in d.get("requests", [])}
        self.snapshots = {(e["name"], e["height"]): [tuple(o) for o in e["owners"]] for e in d.get("snapshots", [])}
        for e in d.get("distributions", []):
            r = RewardSnapshot(**e)
            self.distributions[r.hash()] = r
        self.batch_txids = {(bytes.fromhex(h), b): bytes.fromhex(t) for h, b, t in d.get("batches", [])}

    def save(self) -> None:
        if not self.path:
            return
        with self.lock:
            d = {"requests": sorted(self.requests),
                 "snapshots": [{"name": n, "height": h, "owners": o} for (n, h), o in self.snapshots.items()],
                 "distributions": [r.to_json() for r in self.distributions.values()],
                 "batches": [[h.hex(), b, t.hex()] for (h, b), t in self.batch_txids.items()]}
        tmp = self.path + ".new"
        with open(tmp, "w") as f:
            json.dump(d, f)
        os.replace(tmp, self.path)

    # ------------------------------------------------------------------ snapshot requests
    def schedule(self, name: str, height: int) -> None:
        with self.lock:
            self.requests.add((name, height))
        self.save()

    def cancel(self, name: str, height: int) -> bool:
        with self.lock:
            if (name, height) not in self.requests:
                return False
            self.requests.discard((name, height))
        self.save()
        return True

    def list_requests(self, name: str = "", height: int = 0) -> list[tuple[str, int]]:
        """RetrieveSnapshotRequestsForHeight: std::set order (height-and-name key)."""
        with self.lock:
            rows = [(n, h) for n, h in self.requests if (height == 0 or h == height) and (not name or n == name)]
        return sorted(rows, key=lambda r: (str(r[1]) + r[0]))

    def purge_snapshot(self, name: str, height: int) -> bool:
        with self.lock:
            found = self.snapshots.pop((name, height), None) is not None
        if found:
            self.save()
        return found

    def _address(self, h160: bytes) -> str:
        p = self.state.params
        return _core.base58check_encode(bytes([p.pubkey_prefix]) + h160)

    def take_snapshot(self, name: str, height: int) -> bool:
        owners = sorted((self._address(h), amt) for n, h, amt in self.state.assets.balances() if n == name and amt > 0)
        if not owners:
            log.log_print("rewards", f"no owners exist for asset '{name}' at height {height}")
            return False
        with self.lock:
            self.snapshots[(name, height)] = owners
        return True

    # ------------------------------------------------------------------ block hooks
    def connect_tip(self, block, index, undo: bytes) -> None:
        due = [(n, h) for n, h in self.list_requests("", index.height)]
        if due:
            for n, h in due:
                self.take_snapshot(n, h)
            self.save()

    def block_connected(self, block, index) -> None:
        """CheckRewardDistributions after the tip moved (the pool already reflects the block)."""
        for r in list(self.distributions.values()):
            try:
                self.distribute(r)
            except Exception as e:  # a distribution must never break block processing
                log.log_print("rewards", f"distribution {r.owner_asset}/{r.dist_asset} failed: {e}")

    # ------------------------------------------------------------------ distributions
    def add_distribution(self, r: RewardSnapshot) -> bool:
        h = r.hash()
        with self.lock:
            if h in self.distributions:
                return False
            self.distributions[h] = r
        self.save()
        return True

    def find(self, r: RewardSnapshot) -> RewardSnapshot | None:
        return self.distributions.get(r.hash())

    def _burn_addresses(self) -> set[str]:
        return {addr for addr, _ in _core.asset_burn_info(self.state.params).values()}

    def distribution_list(self, r: RewardSnapshot) -> list[tuple[str, int]] | None:
        """GenerateDistributionList (src/assets/rewards.cpp:44)."""
        st = self.state
        units = 8
        if r.dist_asset != "CLORE":
            meta = st.assets.get(r.dist_asset)
            if meta is None:
                return None
            units = meta["units"]
        scale = 10 ** (8 - units)
        payment = r.amount // scale if r.dist_asset != "CLORE" else r.amount
        if st.assets.get(r.owner_asset) is None:
            return None
        owners = self.snapshots.get((r.owner_asset, r.height))
        if owners is None:
            return None
        skip = set(r.exceptions.split(",")) | self._burn_addresses()
        eligible = sorted((a, amt) for a, amt in owners if a not in skip)
        total = sum(amt for _, amt in eligible)
        if not eligible or total <= 0:
            return None
        out = []
        for addr, owned in eligible:
            reward = (owned * payment * scale // total) // scale * scale
            if reward > 0:
                out.append((addr, reward))
        return out

    def _set_status(self, r: RewardSnapshot, status: int) -> None:
        r.status = status
        self.save()

    def _depth(self, txid: bytes) -> int | None:
        hist = getattr(self.wallet, "history", None)
        w = hist.txs.get(txid) if hist is not None else None
        if w is None:
            return None
        if w.block is None and txid not in self.state.mempool:
            return -1
        return hist.confirmations(w)

    def distribute(self, r: RewardSnapshot) -> None:
        """DistributeRewardSnapshot (src/assets/rewards.cpp:181)."""
        if self.wallet is None or self.wallet.locked:
            return
        payments = self.distribution_list(r)
        if payments is None:
            return
        h = r.hash()
        n_batches = len(payments) // MAX_PAYMENTS_PER_TRANSACTION + 1
        all_confirmed = True
        for i in range(n_batches):
            txid = self.batch_txids.get((h, i))
            if txid is not None:
                depth = self._depth(txid)
                if depth is None or depth > 0:
                    continue
                return  # in the pool (0) or conflicted (<0): wait
            all_confirmed = False
            txid = self._build(r, payments[i * MAX_PAYMENTS_PER_TRANSACTION:(i + 1) * MAX_PAYMENTS_PER_TRANSACTION])
            if txid is None:
                return
            with self.lock:
                self.batch_txids[(h, i)] = txid
            if r.status != PROCESSING:
                r.status = PROCESSING
            self.save()
        if all_confirmed and r.status != COMPLETE:
            self._set_status(r, COMPLETE)

    def _build(self, r: RewardSnapshot, batch: list[tuple[str, int]]) -> bytes | None:
        """BuildTransaction (src/assets/rewards.cpp:246): one transaction paying this batch."""
        p = self.state.params
        w = self.wallet
        total = sum(v for _, v in batch)
        if not batch:
            return None
        if r.dist_asset == "CLORE":
            balance = w.balance(1)
            if total > balance:
                self._set_status(r, LOW_FUNDS)
                return None
            outs = [(_core.address_to_script(a, p.pubkey_prefix, p.script_prefix), v) for a, v in batch]
            try:
                tx, fee = w.create_transaction(outs, fee_rate=w.fee_rate)
            except WalletError:
                self._set_status(r, NOT_ENOUGH_FEE if total >= balance else FAILED_CREATE_TRANSACTION)
                return None
        else:
            aw = self._asset_wallet()
            if sum(u["qty"] for u in aw.unspent(r.dist_asset)) < total:
                self._set_status(r, LOW_REWARDS)
                return None
            try:
                tx = aw.build_transfer_many(r.dist_asset, [(aw._h160(a), v) for a, v in batch])
            except WalletError:
                self._set_status(r, FAILED_CREATE_TRANSACTION)
                return None
        ok, reason, _ = self.state.accept_to_mempool(tx)
        if not ok:
            log.log_print("rewards", f"distribution transaction rejected: {reason}")
            self._set_status(r, FAILED_COMMIT_TRANSACTION)
            return None
        if getattr(w, "history", None) is not None:
            w.history.add(tx)
        return tx.txid()
