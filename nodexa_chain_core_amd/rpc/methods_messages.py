"""Messaging and rewards JSON-RPC methods.

Messages (src/rpc/messages.cpp:490-503): viewallmessages, viewallmessagechannels,
subscribetochannel, unsubscribefromchannel, sendmessage, viewmytaggedaddresses,
viewmyrestrictedaddresses, clearmessages.
Rewards (src/rpc/rewards.cpp:484-495): requestsnapshot, getsnapshotrequest, listsnapshotrequests,
cancelsnapshotrequest, distributereward, getdistributestatus; plus getsnapshot / purgesnapshot
(src/rpc/assets.cpp:2926-3033).

The reference gates the rewards calls behind -assetindex because its owner lists live in an
optional LevelDB index; here the per-address asset balances are always resident in the asset
state (csrc/chain/assets.cpp), so the calls always work.
"""
from __future__ import annotations

import time

from .. import core
from ..wallet import WalletError
from ..wallet.messages import STATUS_NAMES
from ..wallet.rewards import RewardSnapshot
from .protocol import (RPC_DATABASE_ERROR, RPC_INVALID_PARAMETER, RPC_INVALID_PARAMS, RPC_INVALID_REQUEST,
                       RPC_METHOD_NOT_FOUND, RPC_MISC_ERROR, RPC_WALLET_ERROR, RPC_WALLET_INSUFFICIENT_FUNDS,
                       RPCError)

_core = core()
COIN = 100_000_000
MESSAGING_DISABLED = ("Messaging is disabled. To enable messaging, run the wallet without -disablemessaging or "
                      "remove disablemessaging from your clore.conf")


def _date(t: int) -> str:
    """DateTimeStrFormat("%Y-%m-%d %H:%M:%S", t) in UTC."""
    return time.strftime("%Y-%m-%d %H:%M:%S", time.gmtime(t))


def check_ipfs_txid_message(msg: str, expire: int, messages_active: bool) -> None:
    """CheckIPFSTxidMessage (src/rpc/server.cpp:650)."""
    n = len(msg)
    if n in (46, 64):
        if n == 64 and not messages_active:
            raise RPCError(RPC_INVALID_PARAMS, "Invalid txid hash, only ipfs hashes available until HIP5 is activated")
    elif n:
        raise RPCError(RPC_INVALID_PARAMS,
                       "Invalid IPFS hash (must be 46 characters), Txid hashes (must be 64 characters)")
    not_ipfs = msg[:2] != "Qm"
    if not_ipfs and not messages_active:
        raise RPCError(RPC_INVALID_PARAMS, "Invalid ipfs hash. Please use a valid ipfs hash. They usually start with Qm")
    if not_ipfs:
        try:
            bytes.fromhex(msg)
        except ValueError:
            raise RPCError(RPC_INVALID_PARAMS, "Invalid IPFS/Txid hash")
    if expire < 0:
        raise RPCError(RPC_INVALID_PARAMS, "Expire time must be a positive number")


def register(table, node) -> None:
    st = node.state

    def store():
        s = getattr(node, "messages", None)
        if s is None or not s.enabled:
            return None
        return s

    def rewards():
        r = getattr(node, "rewards", None)
        if r is None:
            raise RPCError(RPC_METHOD_NOT_FOUND, "Method not found (wallet disabled)")
        return r

    def _arg(p, i, default=None):
        return p[i] if len(p) > i and p[i] is not None else default

    def _flags():
        return st.asset_flags(st.coins_tip())

    def _channel_name(name: str) -> str:
        kind = _core.asset_name_type(name)[0]
        if kind == "INVALID":
            raise RPCError(RPC_INVALID_PARAMETER, "Channel Name is not valid.")
        if kind in ("ROOT", "SUB"):
            name += "!"
            kind = _core.asset_name_type(name)[0]
            if kind == "INVALID":
                raise RPCError(RPC_INVALID_PARAMETER, "Channel Name is not valid.")
        if kind not in ("OWNER", "MSGCHANNEL"):
            raise RPCError(RPC_INVALID_PARAMETER, "Channel Name must be a owner asset, or a message channel asset "
                                                  "e.g OWNER!, MSG_CHANNEL~123.")
        return name

    # ------------------------------------------------------------------ messages
    def rpc_viewallmessages(p):
        s = store()
        if s is None:
            return MESSAGING_DISABLED
        out = []
        for m in s.view_messages():
            e = {"Asset Name": m.name, "Message": _core.encode_asset_data(m.payload), "Time": _date(m.time),
                 "Block Height": m.height, "Status": STATUS_NAMES.get(m.status, "ERROR")}
            if m.expire:
                try:
                    e["Expire Time"] = _date(m.expire)
                except (OverflowError, OSError, ValueError):
                    e["Expire UTC Time"] = m.expire
            out.append(e)
        return out

    def rpc_viewallmessagechannels(p):
        s = store()
        if s is None:
            return MESSAGING_DISABLED
        with s.lock:
            return sorted(s.channels)

    def rpc_subscribetochannel(p):
        if len(p) != 1:
            raise RPCError(RPC_INVALID_PARAMETER, 'subscribetochannel "channel_name"')
        s = store()
        if s is None:
            raise RPCError(RPC_DATABASE_ERROR, MESSAGING_DISABLED)
        name = _channel_name(str(p[0]))
        s.subscribe(name)
        return "Subscribed to channel: " + name

    def rpc_unsubscribefromchannel(p):
        if len(p) != 1:
            raise RPCError(RPC_INVALID_PARAMETER, 'unsubscribefromchannel "channel_name"')
        s = store()
        if s is None:
            raise RPCError(RPC_DATABASE_ERROR, MESSAGING_DISABLED)
        name = _channel_name(str(p[0]))
        s.unsubscribe(name)
        return "Unsubscribed from channel: " + name

    def rpc_clearmessages(p):
        s = store()
        if s is None:
            raise RPCError(RPC_DATABASE_ERROR, MESSAGING_DISABLED)
        return f"Erased {s.clear()} Messages from the database and cache"

    def rpc_sendmessage(p):
        if len(p) < 2 or len(p) > 3:
            raise RPCError(RPC_INVALID_PARAMETER, 'sendmessage "channel_name" "ipfs_hash" (expire_time)')
        if getattr(node, "wallet", None) is None:
            raise RPCError(RPC_METHOD_NOT_FOUND, "Method not found (wallet disabled)")
        if node.wallet.locked:
            raise RPCError(-13, "Error: Please enter the wallet passphrase with walletpassphrase first.")
        name, ipfs = str(p[0]), str(p[1])
        expire = int(_arg(p, 2, 0))
        check_ipfs_txid_message(ipfs, expire, _flags().msg_restricted)
        kind, err = _core.asset_name_type(name)
        if kind == "INVALID":
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid asset_name: " + err)
        if kind not in ("MSGCHANNEL", "OWNER", "ROOT", "SUB", "RESTRICTED"):
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid asset_name: Only message channels, root, sub, restricted, "
                                                  "and owner assets are allowed")
        if kind in ("ROOT", "SUB"):
            name += "!"
        elif kind == "RESTRICTED":
            name = name[1:] + "!"
        payload = _core.decode_asset_data(ipfs) if ipfs else b""
        aw = node.asset_wallet_instance()
        try:
            txid = aw.send_message(name, payload, expire)
        except WalletError as e:
            msg = str(e)
            if "doesn't own" in msg or "aren't active" in msg:
                raise RPCError(RPC_INVALID_PARAMETER, msg)
            if "Insufficient" in msg:
                raise RPCError(RPC_WALLET_INSUFFICIENT_FUNDS, msg)
            raise RPCError(RPC_WALLET_ERROR, msg)
        return [txid[::-1].hex()]

    def _my_events(which: str, label: str, on: str, off: str):
        s = getattr(node, "messages", None)
        if s is None:
            raise RPCError(RPC_DATABASE_ERROR, "My restricted database is not available")
        with s.lock:
            rows = sorted(getattr(s, which).items())
        out = []
        for (h, name), (flag, t) in rows:
            e = {"Address": node.wallet.address_of(h) if node.wallet else h.hex(), label: name}
            e[on if flag else off] = _date(t)
            out.append(e)
        return out

    def rpc_viewmytaggedaddresses(p):
        return _my_events("my_tags", "Tag Name", "Assigned", "Removed")

    def rpc_viewmyrestrictedaddresses(p):
        return _my_events("my_restricted", "Asset Name", "Restricted", "Derestricted")

    # ------------------------------------------------------------------ rewards
    def _ownership_asset(name: str) -> None:
        kind = _core.asset_name_type(name)[0]
        if kind == "INVALID":
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid asset_name: Please use a valid asset name")
        if kind in ("UNIQUE", "OWNER", "MSGCHANNEL"):
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid asset_name: OWNER, UNQIUE, MSGCHANNEL assets are not "
                                                  "allowed for this call")

    def rpc_requestsnapshot(p):
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'requestsnapshot "asset_name" block_height')
        name, height = str(p[0]), int(p[1])
        _ownership_asset(name)
        if st.assets.get(name) is None:
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid asset_name: asset does not exist.")
        if height <= st.height():
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid block_height: block height should be greater than current "
                                                  "active chain height")
        rewards().schedule(name, height)
        return {"request_status": "Added"}

    def rpc_getsnapshotrequest(p):
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'getsnapshotrequest "asset_name" block_height')
        name, height = str(p[0]), int(p[1])
        if (name, height) in rewards().requests:
            return {"asset_name": name, "block_height": height}
        raise RPCError(RPC_MISC_ERROR, "Failed to retrieve specified snapshot request")

    def rpc_listsnapshotrequests(p):
        if len(p) > 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'listsnapshotrequests ["asset_name" [block_height]]')
        rows = rewards().list_requests(str(_arg(p, 0, "")), int(_arg(p, 1, 0)))
        return [{"asset_name": n, "block_height": h} for n, h in rows]

    def rpc_cancelsnapshotrequest(p):
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'cancelsnapshotrequest "asset_name" block_height')
        if rewards().cancel(str(p[0]), int(p[1])):
            return {"request_status": "Removed"}
        raise RPCError(RPC_MISC_ERROR, "Failed to remove specified snapshot request")

    def _reward_args(p) -> RewardSnapshot:
        name, height, dist = str(p[0]), int(p[1]), str(p[2])
        try:
            amount = round(float(p[3]) * COIN)
        except (TypeError, ValueError):
            raise RPCError(-3, "Amount is not a number or string")
        if amount < 0:
            raise RPCError(-3, "Amount out of range")
        return RewardSnapshot(name, dist, str(_arg(p, 4, "")), amount, height)

    def rpc_distributereward(p):
        if len(p) < 4:
            raise RPCError(RPC_INVALID_PARAMETER, 'distributereward "asset_name" snapshot_height '
                                                  '"distribution_asset_name" gross_distribution_amount '
                                                  '( "exception_addresses" ) ( "change_address" )')
        rw = rewards()
        w = node.wallet
        if w.locked:
            raise RPCError(-13, "Error: Please enter the wallet passphrase with walletpassphrase first.")
        r = _reward_args(p)
        change = str(_arg(p, 5, ""))
        if change and _core.address_to_script(change, node.params.pubkey_prefix, node.params.script_prefix) is None:
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid change address: Use a valid CLORE address")
        _ownership_asset(r.owner_asset)
        if r.height > st.height():
            raise RPCError(RPC_INVALID_PARAMETER, "Invalid snapshot_height: block height should be less than or equal "
                                                  "to the current active chain height")
        if r.dist_asset != "CLORE":
            kind = _core.asset_name_type(r.dist_asset)[0]
            if kind == "INVALID":
                raise RPCError(RPC_INVALID_PARAMETER, "Invalid distribution_asset_name: Please use a valid asset name")
            if kind in ("UNIQUE", "OWNER", "MSGCHANNEL"):
                raise RPCError(RPC_INVALID_PARAMETER, "Invalid distribution_asset_name: OWNER, UNQIUE, MSGCHANNEL "
                                                      "assets are not allowed for this call")
            if not node.asset_wallet_instance().unspent(r.dist_asset + "!"):
                raise RPCError(RPC_INVALID_REQUEST, "Wallet doesn't have the ownership token(!) for the distribution "
                                                    "asset")
        if st.height() - r.height < rw.min_reward_height:
            raise RPCError(RPC_INVALID_REQUEST, "For security of the rewards payout, it is recommended to wait until "
                                                "chain is 60 blocks ahead of the snapshot height. You can modify this "
                                                "by using the -minrewardsheight.")
        if st.assets.get(r.owner_asset) is None:
            raise RPCError(RPC_INVALID_REQUEST, "The asset hasn't been created: " + r.owner_asset)
        if (r.owner_asset, r.height) not in rw.requests:
            raise RPCError(RPC_INVALID_REQUEST, "Snapshot request not found")
        if not rw.add_distribution(r):
            raise RPCError(RPC_INVALID_REQUEST, "Distribution of reward has already be created. You must remove the "
                                                "distribution before creating another one")
        with st.lock:
            rw.distribute(r)
        return "Created reward distribution"

    def rpc_getdistributestatus(p):
        if len(p) < 4:
            raise RPCError(RPC_INVALID_PARAMETER, 'getdistributestatus "asset_name" snapshot_height '
                                                  '"distribution_asset_name" gross_distribution_amount '
                                                  '( "exception_addresses" )')
        r = rewards().find(_reward_args(p))
        if r is None:
            return "Distribution not found"
        return {"Asset Name": r.owner_asset, "Height": str(r.height), "Distribution Name": r.dist_asset,
                "Distribution Amount": r.amount / COIN, "Status": r.status}

    def rpc_getsnapshot(p):
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'getsnapshot "asset_name" block_height')
        name, height = str(p[0]), int(p[1])
        owners = rewards().snapshots.get((name, height))
        if owners is None:
            return None
        return {"name": name, "height": height,
                "owners": [{"address": a, "amount_owned": amt / COIN} for a, amt in owners]}

    def rpc_purgesnapshot(p):
        if len(p) < 2:
            raise RPCError(RPC_INVALID_PARAMETER, 'purgesnapshot "asset_name" block_height')
        name, height = str(p[0]), int(p[1])
        if not rewards().purge_snapshot(name, height):
            return None
        out = {"name": name}
        if height > 0:
            out["height"] = height
        return out

    for cat, name, fn, args in [
        ("messages", "viewallmessages", rpc_viewallmessages, ()),
        ("messages", "viewallmessagechannels", rpc_viewallmessagechannels, ()),
        ("messages", "subscribetochannel", rpc_subscribetochannel, ("channel_name",)),
        ("messages", "unsubscribefromchannel", rpc_unsubscribefromchannel, ("channel_name",)),
        ("messages", "sendmessage", rpc_sendmessage, ("channel", "ipfs_hash", "expire_time")),
        ("restricted", "viewmytaggedaddresses", rpc_viewmytaggedaddresses, ()),
        ("restricted", "viewmyrestrictedaddresses", rpc_viewmyrestrictedaddresses, ()),
        ("messages", "clearmessages", rpc_clearmessages, ()),
        ("rewards", "requestsnapshot", rpc_requestsnapshot, ("asset_name", "block_height")),
        ("rewards", "getsnapshotrequest", rpc_getsnapshotrequest, ("asset_name", "block_height")),
        ("rewards", "listsnapshotrequests", rpc_listsnapshotrequests, ("asset_name", "block_height")),
        ("rewards", "cancelsnapshotrequest", rpc_cancelsnapshotrequest, ("asset_name", "block_height")),
        ("rewards", "distributereward", rpc_distributereward, ("asset_name", "snapshot_height",
                                                               "distribution_asset_name", "gross_distribution_amount",
                                                               "exception_addresses", "change_address")),
        ("rewards", "getdistributestatus", rpc_getdistributestatus, ("asset_name", "block_height",
                                                                     "distribution_asset_name",
                                                                     "gross_distribution_amount",
                                                                     "exception_addresses")),
        ("assets", "getsnapshot", rpc_getsnapshot, ("asset_name", "block_height")),
        ("assets", "purgesnapshot", rpc_purgesnapshot, ("asset_name", "block_height")),
    ]:
        table.append(cat, name, fn, args)
