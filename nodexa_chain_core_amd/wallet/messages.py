"""Asset messaging: channel subscriptions, the message store, and the wallet's tag / restriction
history (SURVEY S10 messaging, A5 "messages" RPC family).

Parity (behaviour):
* CMessage / MessageStatus and the dirty-cache store of src/assets/messages.{h,cpp} — a message is
  the (ipfs hash or txid) payload of an owner-token (`NAME!`) or message-channel (`NAME~CHAN`)
  transfer that goes back to the address the token was spent from, and is kept only when the node
  is subscribed to that channel (src/consensus/tx_verify.cpp:719-737, src/validation.cpp:10517-10532);
  disconnecting its block marks it ORPHAN (src/validation.cpp:9760-9768).
* Automatic subscription on receipt (src/coins.cpp:282-329): owner tokens and channels the wallet
  receives or creates; the owner channel of a ROOT / SUB asset the first time it reaches a wallet
  address that had never received one (the "seen address" spam guard).
* CMyRestrictedDB (src/assets/myrestricteddb.cpp via src/validation.cpp:10534-10548): the latest
  tag / untag and freeze / unfreeze of each wallet address, with the block time.

Everything is resident and persisted as one JSON document (`<datadir>/messages.json`, replaced
atomically) in place of the reference's three LevelDB databases. The hooks run inside
ConnectTip / DisconnectTip (chain/state.ValidationInterface.connect_tip), so the spent coins come
from the block's own undo data.
"""
from __future__ import annotations

import json
import os
import threading
import time
from dataclasses import dataclass

from .. import core
from ..chain.state import ValidationInterface

_core = core()
COIN = 100_000_000

READ, UNREAD, EXPIRED, SPAM, HIDDEN, ORPHAN, MSG_ERROR = range(7)
STATUS_NAMES = {READ: "READ", UNREAD: "UNREAD", EXPIRED: "EXPIRED", SPAM: "SPAM", HIDDEN: "HIDDEN",
                ORPHAN: "ORPHAN", MSG_ERROR: "ERROR"}


@dataclass
class Message:
    txid: bytes
    n: int
    name: str
    payload: bytes      # raw ipfs multihash (34 bytes) or txid (32 bytes)
    time: int           # block time
    expire: int
    height: int = 0
    status: int = UNREAD

    def key(self) -> tuple[bytes, int]:
        return (self.txid, self.n)

    def zmq_json(self) -> str:
        """CZMQMessage::createJsonString (src/assets/messages.cpp:335), byte for byte."""
        return ('{"blockheight": %d, "assetname": "%s", "ipfshash": "%s", "expiretime": %d}'
                % (self.height, self.name, _core.encode_asset_data(self.payload), self.expire))


def is_message_channel(name: str) -> bool:
    return _core.asset_name_type(name)[0] in ("OWNER", "MSGCHANNEL")


class MessageStore(ValidationInterface):
    def __init__(self, state, wallet, path: str | None, enabled: bool = True):
        self.state = state
        self.wallet = wallet
        self.path = path
        self.enabled = enabled  # -disablemessaging turns this off
        self.lock = threading.RLock()
        self.channels: set[str] = set()
        self.seen: set[bytes] = set()  # hash160s that already received an asset (spam guard)
        self.messages: dict[tuple[bytes, int], Message] = {}
        # (hash160, name) -> (flag, block time): latest tag / restriction event of a wallet address
        self.my_tags: dict[tuple[bytes, str], tuple[int, int]] = {}
        self.my_restricted: dict[tuple[bytes, str], tuple[int, int]] = {}
        if path and os.path.exists(path):
            self._load()

    # ------------------------------------------------------------------ persistence
    def _load(self) -> None:
        with open(self.path) as f:
            d = json.load(f)
        self.channels = set(d.get("channels", []))
        self.seen = {bytes.fromhex(h) for h in d.get("seen", [])}
        for e in d.get("messages", []):
            m = Message(bytes.fromhex(e["txid"]), e["n"], e["name"], bytes.fromhex(e["payload"]), e["time"],
                        e["expire"], e["height"], e["status"])
            self.messages[m.key()] = m
        for key, dst in (("tags", self.my_tags), ("restricted", self.my_restricted)):
            for h, name, flag, t in d.get(key, []):
                dst[(bytes.fromhex(h), name)] = (flag, t)

    def save(self) -> None:
        if not self.path:
            return
        with self.lock:
            d = {"channels": sorted(self.channels), "seen": sorted(h.hex() for h in self.seen),
                 "messages": [{"txid": m.txid.hex(), "n": m.n, "name": m.name, "payload": m.payload.hex(),
                               "time": m.time, "expire": m.expire, "height": m.height, "status": m.status}
                              for m in self.messages.values()],
                 "tags": [[h.hex(), n, f, t] for (h, n), (f, t) in self.my_tags.items()],
                 "restricted": [[h.hex(), n, f, t] for (h, n), (f, t) in self.my_restricted.items()]}
        tmp = self.path + ".new"
        with open(tmp, "w") as f:
            json.dump(d, f)
        os.replace(tmp, self.path)

    # ------------------------------------------------------------------ channels
    def is_subscribed(self, name: str) -> bool:
        with self.lock:
            return name in self.channels

    def subscribe(self, name: str) -> None:
        with self.lock:
            self.channels.add(name)
        self.save()

    def unsubscribe(self, name: str) -> None:
        with self.lock:
            self.channels.discard(name)
        self.save()

    def view_messages(self) -> list[Message]:
        """std::set<CMessage> order: by outpoint (txid bytes, then output index)."""
        with self.lock:
            return [self.messages[k] for k in sorted(self.messages)]

    def clear(self) -> int:
        with self.lock:
            n = len(self.messages)
            self.messages.clear()
        self.save()
        return n

    # ------------------------------------------------------------------ block hooks
    def _mine(self, spk: bytes) -> bool:
        return self.wallet is not None and self.wallet.is_mine(spk)

    def _auto_subscribe(self, a: dict, spk: bytes) -> bool:
        """AddCoins' subscription rules (src/coins.cpp:282-329). Returns True if anything changed."""
        kind = _core.asset_name_type(a["name"])[0]
        before = (len(self.channels), len(self.seen))
        if a["type"] == "transfer_asset" and a["amount"] > 0 and self._mine(spk):
            if kind in ("ROOT", "SUB"):
                owner = _core.asset_parent_name(a["name"]) + "!"
                if owner not in self.channels and a["hash160"] not in self.seen:
                    self.channels.add(owner)
                    self.seen.add(a["hash160"])
            elif kind in ("OWNER", "MSGCHANNEL"):
                self.channels.add(a["name"])
                self.seen.add(a["hash160"])
        elif a["type"] in ("new_asset", "owner"):
            if self._mine(spk):
                if kind in ("ROOT", "SUB"):
                    self.channels.add(a["name"] + "!")
                    self.seen.add(a["hash160"])
                elif kind in ("OWNER", "MSGCHANNEL"):
                    self.channels.add(a["name"])
                    self.seen.add(a["hash160"])
            elif kind == "MSGCHANNEL" and _core.asset_parent_name(a["name"]) + "!" in self.channels:
                self.channels.add(a["name"])
        return (len(self.channels), len(self.seen)) != before

    def connect_tip(self, block, index, undo: bytes) -> None:
        if not self.enabled:
            return
        prev = self.state.chain.find(index.prev_hash)
        flags = self.state.asset_flags(prev) if prev is not None else None
        if flags is None or not flags.assets:
            return
        changed = False
        now = int(time.time())
        found: list[Message] = []
        with self.lock:
            for t, tx in enumerate(block.vtx):
                parsed = [(_core.parse_asset_script(o.script_pubkey), o.script_pubkey) for o in tx.vout]
                if self.wallet is not None:
                    for a, spk in parsed:
                        if a is not None:
                            changed |= self._auto_subscribe(a, spk)
                if t > 0 and flags.msg_restricted:
                    found += self._messages_of(tx, t, parsed, undo, block.header.time, index.height, now)
                    changed |= self._restriction_events(tx, block.header.time)
            for m in found:
                if m.expire == 0 or now < m.expire:
                    self.state._emit("new_asset_message", m)
                if m.name in self.channels:
                    self.messages[m.key()] = m
                    changed = True
        if changed:
            self.save()

    def _messages_of(self, tx, t: int, parsed, undo: bytes, block_time: int, height: int, now: int) -> list[Message]:
        cands = [(n, a) for n, (a, _) in enumerate(parsed)
                 if a is not None and a["type"] == "transfer_asset" and a["message"]
                 and is_message_channel(a["name"]) and (a["expire"] == 0 or a["expire"] > now)]
        if not cands:
            return []
        spent_from: dict[str, bytes] = {}  # asset name -> address of the first input carrying it
        for i in range(len(tx.vin)):
            _, spk, _, _ = _core.block_undo_coin(undo, t, i)
            a = _core.parse_asset_script(spk)
            if a is not None and a["name"] not in spent_from:
                spent_from[a["name"]] = a["hash160"]
        txid = tx.txid()
        return [Message(txid, n, a["name"], a["message"], block_time, a["expire"], height)
                for n, a in cands if spent_from.get(a["name"]) == a["hash160"]]

    def _restriction_events(self, tx, block_time: int) -> bool:
        changed = False
        for o in tx.vout:
            d = _core.parse_null_asset_script(o.script_pubkey)
            if d is None or d["type"] != "tag" or self.wallet is None:
                continue
            if d["hash160"] not in self.wallet.keys:
                continue
            kind = _core.asset_name_type(d["name"])[0]
            if kind in ("QUALIFIER", "SUB_QUALIFIER"):
                self.my_tags[(d["hash160"], d["name"])] = (d["flag"], block_time)
                changed = True
            elif kind == "RESTRICTED":
                self.my_restricted[(d["hash160"], d["name"])] = (d["flag"], block_time)
                changed = True
        return changed

    def disconnect_tip(self, block, index, undo: bytes) -> None:
        if not self.enabled:
            return
        changed = False
        with self.lock:
            for tx in block.vtx[1:]:
                txid = tx.txid()
                for n, o in enumerate(tx.vout):
                    a = _core.parse_asset_script(o.script_pubkey)
                    if a is None or a["type"] != "transfer_asset" or not a["message"]:
                        continue
                    m = self.messages.get((txid, n))
                    if m is not None and a["name"] in self.channels:
                        m.status = ORPHAN
                        changed = True
        if changed:
            self.save()
