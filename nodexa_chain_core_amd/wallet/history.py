"""Wallet transaction history (CWalletTx bookkeeping).

Parity (behaviour): CWallet::AddToWalletIfInvolvingMe / SyncTransaction (src/wallet/wallet.cpp) —
every transaction that pays a wallet script or spends a wallet output is recorded with the block
that confirmed it (or none while in the pool); ListTransactions / GetAmounts (credit, debit, fee,
categories send / receive / generate / immature / orphan) drive listtransactions, gettransaction,
listsinceblock, getreceivedbyaddress and listreceivedbyaddress (src/wallet/rpcwallet.cpp).
Records live in <datadir>/wallet_txs.json (the role of the wallet database's "tx" records),
rewritten atomically once per connected block / wallet send.
"""
from __future__ import annotations

import json
import os
import threading
import time

from .. import core
from ..chain.state import ValidationInterface

_core = core()
COIN = 100_000_000


class WalletTx:
    __slots__ = ("tx", "time", "block", "abandoned", "comment", "order", "comment_to", "from_account",
                 "replaced_by", "replaces")

    def __init__(self, tx, t: int, block: bytes | None = None, order: int = 0):
        self.tx, self.time, self.block = tx, t, block
        self.abandoned = False
        self.comment = ""
        self.order = order  # nOrderPos: insertion order
        self.comment_to = ""
        self.from_account = None  # strFromAccount (sendfrom)
        self.replaced_by = None   # bumpfee bookkeeping (mapValue "replaced_by_txid" / "replaces_txid")
        self.replaces = None


class WalletHistory(ValidationInterface):
    def __init__(self, wallet, path: str | None):
        self.w = wallet
        self.on_change = None  # callable(txid) for -walletnotify
        self.state = wallet.state
        self.path = path
        self.lock = threading.RLock()
        self.txs: dict[bytes, WalletTx] = {}
        self.locked: set[tuple[bytes, int]] = set()  # lockunspent
        self.moves: list[tuple] = []  # CAccountingEntry: (account, amount, time, other_account, comment)
        if path and os.path.exists(path):
            self._load()

    # ------------------------------------------------------------------ persistence
    def _load(self) -> None:
        with open(self.path) as f:
            d = json.load(f)
        for h, e in d.get("txs", {}).items():
            wtx = WalletTx(_core.Transaction.deserialize(bytes.fromhex(e["hex"])), e["time"],
                           bytes.fromhex(e["block"]) if e.get("block") else None)
            wtx.abandoned = e.get("abandoned", False)
            wtx.comment = e.get("comment", "")
            wtx.order = e.get("order", len(self.txs))
            wtx.comment_to = e.get("comment_to", "")
            wtx.from_account = e.get("from_account")
            wtx.replaced_by = bytes.fromhex(e["replaced_by"]) if e.get("replaced_by") else None
            wtx.replaces = bytes.fromhex(e["replaces"]) if e.get("replaces") else None
            self.txs[bytes.fromhex(h)] = wtx
        self.moves = [tuple(m) for m in d.get("moves", [])]

    def save(self) -> None:
        if not self.path:
            return
        with self.lock:
            d = {"txs": {h.hex(): {"hex": w.tx.serialize(True).hex(), "time": w.time,
                                   "block": w.block.hex() if w.block else None, "abandoned": w.abandoned,
                                   "comment": w.comment, "order": w.order, "comment_to": w.comment_to,
                                   "from_account": w.from_account,
                                   "replaced_by": w.replaced_by.hex() if w.replaced_by else None,
                                   "replaces": w.replaces.hex() if w.replaces else None}
                         for h, w in self.txs.items()},
                 "moves": self.moves}
        tmp = self.path + ".new"
        with open(tmp, "w") as f:
            json.dump(d, f)
        os.replace(tmp, self.path)

    # ------------------------------------------------------------------ involvement
    def _ours(self, spk: bytes, watch: bool) -> bool:
        return self.w.is_mine(spk) or (watch and self.w.is_watch(spk))

    def _output_mine(self, prevout, watch: bool = False) -> tuple[int, bytes] | None:
        w = self.txs.get(prevout.hash)
        if w is None or prevout.n >= len(w.tx.vout):
            return None
        o = w.tx.vout[prevout.n]
        return (o.value, o.script_pubkey) if self._ours(o.script_pubkey, watch) else None

    def involves_me(self, tx) -> bool:
        """IsMine(ISMINE_ALL) of an output or of a spent wallet output (watch-only included)."""
        if any(self._ours(o.script_pubkey, True) for o in tx.vout):
            return True
        return not tx.is_coinbase() and any(self._output_mine(i.prevout, True) for i in tx.vin)

    def involves_watch(self, w: "WalletTx") -> bool:
        tx = w.tx
        if any(self.w.is_watch(o.script_pubkey) for o in tx.vout):
            return True
        return not tx.is_coinbase() and any(
            (m := self._output_mine(i.prevout, True)) is not None and self.w.is_watch(m[1]) for i in tx.vin)

    def remove(self, txid: bytes) -> bool:
        """removeprunedfunds: forget a wallet transaction."""
        with self.lock:
            found = self.txs.pop(txid, None) is not None
        if found:
            self.save()
        return found

    def add(self, tx, block: bytes | None = None, save: bool = True) -> bool:
        txid = tx.txid()
        with self.lock:
            w = self.txs.get(txid)
            new = w is None
            if w is None:
                if not self.involves_me(tx):
                    return False
                w = self.txs[txid] = WalletTx(tx, int(time.time()), order=len(self.txs))
            updated = block is not None and w.block != block
            if block is not None:
                w.block = block
                w.abandoned = False
        if save:
            self.save()
        if (new or updated) and self.on_change is not None:  # AddToWallet -> -walletnotify
            self.on_change(txid)
        return True

    # ValidationInterface
    def transaction_added_to_mempool(self, tx) -> None:
        self.add(tx)

    def block_connected(self, block, index) -> None:
        changed = False
        for tx in block.vtx:
            changed |= self.add(tx, index.hash, save=False)
        if changed:
            self.save()

    # ------------------------------------------------------------------ amounts
    def confirmations(self, w: WalletTx) -> int:
        st = self.state
        if w.block is None:
            return 0 if w.tx.txid() in st.mempool or not w.abandoned else -1
        idx = st.chain.find(w.block)
        if idx is None or not st.chain.in_active_chain(idx):
            return 0
        return st.height() - idx.height + 1

    def debit(self, w: WalletTx, watch: bool = False) -> int:
        if w.tx.is_coinbase():
            return 0
        return sum(m[0] for i in w.tx.vin if (m := self._output_mine(i.prevout, watch)) is not None)

    def credit(self, w: WalletTx, watch: bool = False) -> int:
        return sum(o.value for o in w.tx.vout if self._ours(o.script_pubkey, watch))

    def fee(self, w: WalletTx) -> int | None:
        """Only known when every input is ours (the reference reports fee for fully-from-me txs)."""
        if w.tx.is_coinbase():
            return None
        ins = [self._output_mine(i.prevout) for i in w.tx.vin]
        if any(m is None for m in ins):
            return None
        return sum(m[0] for m in ins) - w.tx.value_out()

    def _address(self, spk: bytes) -> str | None:
        p = self.w.params
        return _core.script_to_address(spk, p.pubkey_prefix, p.script_prefix) or None

    def entries(self, w: WalletTx, watch: bool = False) -> list[dict]:
        """ListTransactions entries of one wallet transaction (sends, then receives); watch-only
        outputs count when `watch` (include_watchonly) and are flagged involvesWatchonly."""
        conf = self.confirmations(w)
        rbf = "no"
        if conf <= 0:
            rbf = "yes" if any(i.sequence <= 0xfffffffd for i in w.tx.vin) else "unknown" if conf < 0 else "no"
        base = {"confirmations": conf, "txid": w.tx.txid()[::-1].hex(), "time": w.time, "timereceived": w.time,
                "bip125-replaceable": rbf, "walletconflicts": []}
        if w.replaced_by:
            base["replaced_by_txid"] = w.replaced_by[::-1].hex()
        if w.replaces:
            base["replaces_txid"] = w.replaces[::-1].hex()
        if w.comment_to:
            base["to"] = w.comment_to
        if w.block is not None:
            idx = self.state.chain.find(w.block)
            if idx is not None:
                base["blockhash"] = w.block[::-1].hex()
                base["blocktime"] = idx.time
                blk = self.state.get_block(w.block)
                if blk is not None:
                    base["blockindex"] = [t.txid() for t in blk.vtx].index(w.tx.txid()) if blk else 0
        if w.comment:
            base["comment"] = w.comment
        out = []
        debit = self.debit(w, watch)
        fee = self.fee(w)
        sends, receives = [], []
        for n, o in enumerate(w.tx.vout):  # GetAmounts: change (mine, no address-book label) is skipped
            mine = self._ours(o.script_pubkey, watch)
            wo = mine and self.w.is_watch(o.script_pubkey)
            if debit > 0:
                if mine and self._is_change(o.script_pubkey):
                    continue
                e = {"account": w.from_account or "", "address": self._address(o.script_pubkey), "category": "send",
                     "amount": -o.value / COIN, "vout": n, "fee": -(fee or 0) / COIN, "abandoned": w.abandoned}
                if wo:
                    e["involvesWatchonly"] = True
                e.update(base)
                sends.append(e)
            if mine:
                cat = "receive"
                if w.tx.is_coinbase():
                    cat = "orphan" if conf <= 0 else ("immature" if conf <= _core.COINBASE_MATURITY else "generate")
                e = {"account": self._label(o.script_pubkey), "address": self._address(o.script_pubkey),
                     "category": cat, "amount": o.value / COIN, "vout": n}
                if wo:
                    e["involvesWatchonly"] = True
                e.update(base)
                receives.append(e)
        out = sends + receives
        return out

    def _is_change(self, spk: bytes) -> bool:
        return len(spk) == 25 and self.w.labels.get(spk[3:23]) == "change"

    def _label(self, spk: bytes) -> str:
        if spk in self.w.watch:
            return self.w.watch[spk].get("label", "")
        return self.w.labels.get(spk[3:23], "") if len(spk) == 25 else ""

    def ordered(self) -> list[WalletTx]:
        with self.lock:
            return sorted(self.txs.values(), key=lambda w: w.order)

    def received_by(self, minconf: int = 1, watch: bool = False) -> dict[bytes, tuple[int, int, list[str]]]:
        """scriptPubKey -> (amount, min confirmations, txids) over non-coinbase wallet txs."""
        out: dict[bytes, list] = {}
        for w in self.ordered():
            if w.tx.is_coinbase():
                continue
            conf = self.confirmations(w)
            if conf < minconf:
                continue
            for o in w.tx.vout:
                if self._ours(o.script_pubkey, watch):
                    e = out.setdefault(o.script_pubkey, [0, 1 << 30, []])
                    e[0] += o.value
                    e[1] = min(e[1], conf)
                    e[2].append(w.tx.txid()[::-1].hex())
        return {k: (v[0], v[1], v[2]) for k, v in out.items()}
