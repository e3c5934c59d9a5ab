"""Asset messaging (channel subscriptions, message store, orphaning on disconnect, my tagged
addresses) and reward snapshots / distributions, modelled on the reference's
test/functional/feature_messaging.py and feature_rewards.py flows. Node B follows node A by
submitblock so each node keeps its own wallet and message store."""
import hashlib
import struct

import pytest

from test_node_rpc import client
from test_p2p import _node

IPFS = "QmZPGfJojdTzaqCWJu2m3krark38X1rqEHBo4SjeqHKB26"


def _sync(ca, cb):
    for h in range(cb.getblockcount() + 1, ca.getblockcount() + 1):
        assert cb.submitblock(ca.getblock(ca.getblockhash(h), 0)) is None


def _ext(core, seed):
    return core.base58check_encode(bytes([42]) + hashlib.sha256(seed).digest()[:20])


def test_messaging_between_two_wallets(core, tmp_path):
    a = _node(core, tmp_path, "a", [])
    b = _node(core, tmp_path, "b", [])
    try:
        ca, cb = client(a), client(b)
        w = ca.getnewaddress()
        ca.generatetoaddress(432, w)  # assets + messaging_restricted active from 433 on regtest
        with pytest.raises(RuntimeError, match="Wallet doesn't have asset: MESSAGING!"):
            ca.issue("MESSAGING~ONE")
        ca.issue("MESSAGING", 100)
        ca.issue("MESSAGING~ONE")
        ca.issue("MESSAGING~TWO")
        ca.issue("SPAM", 100)
        ca.generatetoaddress(1, w)
        _sync(ca, cb)
        # the issuing wallet is subscribed to its own channels
        assert {"MESSAGING!", "MESSAGING~ONE", "MESSAGING~TWO", "SPAM!"} <= set(ca.viewallmessagechannels())
        assert cb.viewallmessagechannels() == []
        assert cb.subscribetochannel("MESSAGING") == "Subscribed to channel: MESSAGING!"  # ROOT -> owner channel
        cb.subscribetochannel("MESSAGING~ONE")
        assert cb.viewallmessagechannels() == ["MESSAGING!", "MESSAGING~ONE"]
        with pytest.raises(RuntimeError, match="owner asset, or a message channel"):
            cb.subscribetochannel("#KYC")

        ca.sendmessage("MESSAGING!", IPFS)
        ca.generatetoaddress(1, w)
        _sync(ca, cb)
        msgs = cb.viewallmessages()
        assert len(msgs) == 1
        m = msgs[0]
        assert (m["Asset Name"], m["Message"], m["Status"]) == ("MESSAGING!", IPFS, "UNREAD")
        assert m["Block Height"] == cb.getblockcount() and len(m["Time"]) == 19
        assert len(ca.viewallmessages()) == 1  # the sender is subscribed to its own channel
        assert cb.clearmessages() == "Erased 1 Messages from the database and cache"
        assert cb.viewallmessages() == []

        # only subscribed channels are kept; a txid payload and an expiry are carried through
        txid_payload = "ab" * 32
        ca.sendmessage("MESSAGING~ONE", txid_payload, 4_000_000_000)
        ca.sendmessage("MESSAGING~TWO", IPFS)
        ca.generatetoaddress(1, w)
        _sync(ca, cb)
        msgs = cb.viewallmessages()
        assert [(m["Asset Name"], m["Message"]) for m in msgs] == [("MESSAGING~ONE", txid_payload)]
        assert msgs[0]["Expire Time"].startswith("2096-")
        cb.clearmessages()
        cb.unsubscribefromchannel("MESSAGING!")
        cb.unsubscribefromchannel("MESSAGING~ONE")
        assert cb.viewallmessagechannels() == []
        with pytest.raises(RuntimeError, match="Invalid IPFS hash"):
            ca.sendmessage("MESSAGING!", "Qm123")
        with pytest.raises(RuntimeError, match="doesn't own"):
            cb.sendmessage("MESSAGING!", IPFS)

        # auto-subscribe on the first asset a fresh address receives (spam guard afterwards)
        addr1 = cb.getnewaddress()
        ca.transfer("MESSAGING", 10, addr1)
        ca.generatetoaddress(1, w)
        _sync(ca, cb)
        assert cb.viewallmessagechannels() == ["MESSAGING!"]
        ca.transfer("SPAM", 10, addr1)
        ca.generatetoaddress(1, w)
        _sync(ca, cb)
        assert cb.viewallmessagechannels() == ["MESSAGING!"]

        # a message whose block is disconnected becomes ORPHAN
        ca.sendmessage("MESSAGING!", IPFS)
        blk = ca.generatetoaddress(1, w)[0]
        _sync(ca, cb)
        assert [m["Status"] for m in cb.viewallmessages()] == ["UNREAD"]
        cb.invalidateblock(blk)
        assert [m["Status"] for m in cb.viewallmessages()] == ["ORPHAN"]
        cb.reconsiderblock(blk)
        assert cb.getbestblockhash() == blk

        # the wallet's own tag history (viewmytaggedaddresses)
        ca.issuequalifierasset("#KYC", 1)
        ca.generatetoaddress(1, w)
        ca.addtagtoaddress("#KYC", addr1)
        ca.generatetoaddress(1, w)
        _sync(ca, cb)
        tags = cb.viewmytaggedaddresses()
        assert [(t["Address"], t["Tag Name"]) for t in tags] == [(addr1, "#KYC")] and "Assigned" in tags[0]
        assert ca.viewmytaggedaddresses() == []  # addr1 is not A's
        assert cb.viewmyrestrictedaddresses() == []
    finally:
        b.stop()
        a.stop()


def test_message_store_persists_and_disablemessaging(core, tmp_path):
    from nodexa_chain_core_amd.wallet.messages import Message, MessageStore

    class _W:
        keys = {}

        def is_mine(self, spk):
            return False

    path = str(tmp_path / "messages.json")
    s = MessageStore(None, _W(), path)
    s.subscribe("ABC!")
    m = Message(b"\x01" * 32, 3, "ABC!", core.decode_asset_data(IPFS), 1_600_000_000, 0, 7)
    s.messages[m.key()] = m
    s.save()
    s2 = MessageStore(None, _W(), path)
    assert s2.channels == {"ABC!"} and s2.messages[m.key()] == m
    assert m.zmq_json() == ('{"blockheight": 7, "assetname": "ABC!", "ipfshash": "%s", "expiretime": 0}' % IPFS)

    node = _node(core, tmp_path, "off", ["-disablemessaging"])
    try:
        c = client(node)
        assert c.viewallmessages().startswith("Messaging is disabled")
        with pytest.raises(RuntimeError, match="Messaging is disabled"):
            c.subscribetochannel("ABC!")
    finally:
        node.stop()


def test_reward_snapshot_hash_layout():
    from nodexa_chain_core_amd.wallet.rewards import RewardSnapshot

    r = RewardSnapshot("STOCK1", "CLORE", "addr", 2000 * 10**8, 512)
    raw = b"\x06STOCK1\x05CLORE\x04addr" + struct.pack("<qI", 2000 * 10**8, 512)
    assert r.hash() == hashlib.sha256(hashlib.sha256(raw).digest()).digest()
    r.status = 3
    assert r.hash() == RewardSnapshot("STOCK1", "CLORE", "addr", 2000 * 10**8, 512).hash()  # status not hashed


def test_rewards_snapshot_and_distribution(core, tmp_path):
    node = _node(core, tmp_path, "r", ["-minrewardheight=3", "-assetindex"])
    try:
        c = client(node)
        w = c.getnewaddress()
        c.generatetoaddress(432, w)
        owner = c.getnewaddress()
        c.issue("STOCK1", 1000, owner)
        c.issue("PAYOUT", 10000, owner)
        c.generatetoaddress(1, w)
        sh0, sh1 = c.getnewaddress(), c.getnewaddress()
        sh2 = _ext(core, b"sh2")
        c.transfer("STOCK1", 200, sh0, "", 0, "", owner)
        c.generatetoaddress(1, w)
        c.transfer("STOCK1", 300, sh1, "", 0, "", owner)
        c.generatetoaddress(1, w)
        c.transfer("STOCK1", 100, sh2, "", 0, "", owner)
        c.generatetoaddress(1, w)
        assert c.listaddressesbyasset("STOCK1") == {owner: 400, sh0: 200, sh1: 300, sh2: 100}

        h = c.getblockcount() + 2
        with pytest.raises(RuntimeError, match="asset does not exist"):
            c.requestsnapshot("NOPE", h)
        with pytest.raises(RuntimeError, match="OWNER, UNQIUE, MSGCHANNEL"):
            c.requestsnapshot("STOCK1!", h)
        with pytest.raises(RuntimeError, match="greater than current"):
            c.requestsnapshot("STOCK1", c.getblockcount())
        assert c.requestsnapshot("STOCK1", h) == {"request_status": "Added"}
        c.requestsnapshot("STOCK1", h + 50)
        c.requestsnapshot("PAYOUT", h + 50)
        assert c.getsnapshotrequest("STOCK1", h) == {"asset_name": "STOCK1", "block_height": h}
        assert len(c.listsnapshotrequests()) == 3
        assert c.listsnapshotrequests("STOCK1") == [{"asset_name": "STOCK1", "block_height": h},
                                                    {"asset_name": "STOCK1", "block_height": h + 50}]
        assert c.listsnapshotrequests("", h + 50) == [{"asset_name": "PAYOUT", "block_height": h + 50},
                                                      {"asset_name": "STOCK1", "block_height": h + 50}]
        assert c.cancelsnapshotrequest("PAYOUT", h + 50) == {"request_status": "Removed"}
        with pytest.raises(RuntimeError, match="Failed to remove"):
            c.cancelsnapshotrequest("PAYOUT", h + 50)

        c.generatetoaddress(2, w)
        # moving shares after the snapshot height does not change the snapshot
        c.transfer("STOCK1", 100, sh1, "", 0, "", owner)
        c.generatetoaddress(1, w)
        snap = c.getsnapshot("STOCK1", h)
        assert snap["name"] == "STOCK1" and snap["height"] == h
        assert {o["address"]: o["amount_owned"] for o in snap["owners"]} == {owner: 400, sh0: 200, sh1: 300, sh2: 100}
        with pytest.raises(RuntimeError, match="recommended to wait"):
            c.distributereward("STOCK1", h, "CLORE", 1200, owner)
        c.generatetoaddress(2, w)
        with pytest.raises(RuntimeError, match="Snapshot request not found"):
            c.distributereward("PAYOUT", h, "CLORE", 100, owner)
        with pytest.raises(RuntimeError, match="hasn't been created"):
            c.distributereward("GHOST", h, "CLORE", 100, owner)

        # CLORE payout in proportion 200:300:100 over 1200, the owner address excepted
        assert c.distributereward("STOCK1", h, "CLORE", 1200, owner) == "Created reward distribution"
        with pytest.raises(RuntimeError, match="already be created"):
            c.distributereward("STOCK1", h, "CLORE", 1200, owner)
        assert c.getdistributestatus("STOCK1", h, "CLORE", 1200, owner)["Status"] == 1
        c.generatetoaddress(1, w)
        assert c.getreceivedbyaddress(sh0, 1) == 400 and c.getreceivedbyaddress(sh1, 1) == 600
        c.generatetoaddress(1, w)
        st = c.getdistributestatus("STOCK1", h, "CLORE", 1200, owner)
        assert st == {"Asset Name": "STOCK1", "Height": str(h), "Distribution Name": "CLORE",
                      "Distribution Amount": 1200, "Status": 2}
        assert c.getdistributestatus("STOCK1", h, "CLORE", 1, owner) == "Distribution not found"

        # asset payout: 7 indivisible PAYOUT units over 200:300:100 -> 2, 3, 1 (remainder stays)
        c.distributereward("STOCK1", h, "PAYOUT", 7, owner)
        c.generatetoaddress(1, w)
        assert c.listassetbalancesbyaddress(sh0)["PAYOUT"] == 2
        assert c.listassetbalancesbyaddress(sh1)["PAYOUT"] == 3
        assert c.listassetbalancesbyaddress(sh2)["PAYOUT"] == 1
        # too large a CLORE payout: LOW_FUNDS (3), retried every block
        c.distributereward("STOCK1", h, "CLORE", 10_000_000, owner, "")
        assert c.getdistributestatus("STOCK1", h, "CLORE", 10_000_000, owner)["Status"] == 3
        # too large an asset payout: LOW_REWARDS (5)
        c.distributereward("STOCK1", h, "PAYOUT", 20000, owner)
        assert c.getdistributestatus("STOCK1", h, "PAYOUT", 20000, owner)["Status"] == 5
        with pytest.raises(RuntimeError, match="ownership token"):
            c.distributereward("STOCK1", h, "STOCK1/NOPE", 1, owner)
        # transferfromaddresses: only the listed addresses' coins are spent
        before = c.listaddressesbyasset("PAYOUT")
        c.transferfromaddresses("PAYOUT", [sh0], 2, sh2, "", 0, "", sh0)
        c.generatetoaddress(1, w)
        after = c.listaddressesbyasset("PAYOUT")
        assert after.get(sh0, 0) == before[sh0] - 2 and after[sh2] == before[sh2] + 2
        assert sum(after.values()) == sum(before.values())
        assert {a: v for a, v in after.items() if a not in (sh0, sh2)} == \
            {a: v for a, v in before.items() if a not in (sh0, sh2)}
        with pytest.raises(RuntimeError, match="Insufficient asset funds"):
            c.transferfromaddress("PAYOUT", sh1, 100, sh2)
        with pytest.raises(RuntimeError, match="non-empty array"):
            c.transferfromaddresses("PAYOUT", [], 1, sh2)
        assert c.purgesnapshot("STOCK1", h) == {"name": "STOCK1", "height": h}
        assert c.getsnapshot("STOCK1", h) is None
    finally:
        node.stop()
