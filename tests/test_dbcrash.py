"""Chain-state crash consistency and the UTXO statistics that check it.

* gettxoutsetinfo as the reference computes it (GetUTXOStats / ApplyStats,
  /root/reference/src/rpc/blockchain.cpp:1076-1130): hash_serialized_2 over the best block and the
  coins grouped by transaction, bogosize, disk_size of the chainstate store, the flush first —
  re-derived here in Python from the blocks' own outputs, and the reference's
  rpc_blockchain.py invalidate / reconsider round trip (parity unpinned: no reference node runs here);
* feature_dbcrash.py's loop (/root/reference/test/functional/feature_dbcrash.py): a daemon started
  again and again with -dbcrashratio dies in the middle of flushes; every restart must recover, and
  the UTXO set it ends with must equal the one -reindex-chainstate rebuilds from the stored blocks.
"""
import hashlib
import os
import subprocess
import sys

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _varint(n: int) -> bytes:
    out = []
    while True:
        out.append((n & 0x7F) | (0x80 if out else 0))
        if n <= 0x7F:
            break
        n = (n >> 7) - 1
    return bytes(reversed(out))


def _compact(n: int) -> bytes:
    return bytes([n]) if n < 253 else b"\xfd" + n.to_bytes(2, "little")


def _expected_stats(c, height):
    """The UTXO set of a chain of coinbase-only blocks, hashed the reference's way."""
    coins = {}  # txid (storage order) -> (height, [(n, spk, value)])
    for h in range(1, height + 1):
        blk = c.getblock(c.getblockhash(h), 2)
        for tx in blk["tx"]:
            outs = []
            for o in tx["vout"]:
                spk = bytes.fromhex(o["scriptPubKey"]["hex"])
                if spk[:1] == b"\x6a":  # OP_RETURN: IsUnspendable, never a coin
                    continue
                outs.append((o["n"], spk, round(o["value"] * 1e8)))
            if outs:
                coins[bytes.fromhex(tx["txid"])[::-1]] = (h, outs)
    ss = bytes.fromhex(c.getblockhash(height))[::-1]
    bogo = 0
    for txid in sorted(coins):
        h, outs = coins[txid]
        ss += txid + _varint(h * 2 + 1)  # coinbase
        for n, spk, value in sorted(outs):
            ss += _varint(n + 1) + _compact(len(spk)) + spk + _varint(value)
            bogo += 32 + 4 + 4 + 8 + 2 + len(spk)
        ss += _varint(0)
    digest = hashlib.sha256(hashlib.sha256(ss).digest()).digest()[::-1].hex()
    return digest, bogo, sum(len(o) for _, o in coins.values()), len(coins)


def test_gettxoutsetinfo_reference_layout(core, node_factory):  # noqa: F811
    node, addr = node_factory()
    c = client(node)
    c.generatetoaddress(12, addr)
    res = c.gettxoutsetinfo()
    digest, bogo, txouts, ntx = _expected_stats(c, 12)
    assert res["height"] == 12 and res["bestblock"] == c.getblockhash(12)
    assert (res["txouts"], res["transactions"], res["bogosize"]) == (txouts, ntx, bogo)
    assert res["hash_serialized_2"] == digest
    assert res["disk_size"] > 0  # flushed first: the chainstate store holds the set
    # rpc_blockchain.py: genesis-only chain, then the same result after reconsiderblock
    b1 = c.getblockhash(1)
    c.invalidateblock(b1)
    res2 = c.gettxoutsetinfo()
    assert (res2["height"], res2["txouts"], res2["transactions"], res2["bogosize"], res2["total_amount"]) == (0, 0, 0, 0, 0)
    assert res2["bestblock"] == c.getblockhash(0)
    c.reconsiderblock(b1)
    res3 = c.gettxoutsetinfo()
    for k in ("total_amount", "transactions", "height", "txouts", "bogosize", "bestblock", "hash_serialized_2"):
        assert res3[k] == res[k], k


_CHILD = """
import sys
sys.path.insert(0, {root!r})
from nodexa_chain_core_amd.node import Node
from nodexa_chain_core_amd.utils.config import ArgsManager
from nodexa_chain_core_amd.rpc.client import RPCClient
from nodexa_chain_core_amd import _core
a = ArgsManager()
a.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", "-datadir={d}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p", "-printtoconsole=0",
                    "-dbcrashratio={ratio}"])
n = Node(a)
n.start()
c = RPCClient("127.0.0.1", n.rpc.port, "u", "p")
print("start", c.getblockcount(), flush=True)
addr = _core.base58check_encode(bytes([42]) + bytes(range(20)))
for _ in range(3):
    c.generatetoaddress(2, addr)
    c.gettxoutsetinfo()  # FlushStateToDisk: the crash point
n.stop()
print("clean", flush=True)
"""


def test_dbcrash_cycles_then_reindex_chainstate(core, node_factory, tmp_path):  # noqa: F811
    d = tmp_path / "crashy"
    os.makedirs(d)
    heights, crashes = [], 0
    for i in range(6):
        r = subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT, d=d, ratio=2)], capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        starts = [int(x.split()[1]) for x in r.stdout.splitlines() if x.startswith("start")]
        assert len(starts) == 1, (r.stdout, r.stderr[-3000:])  # every restart recovered and served RPC
        heights.append(starts[0])
        crashes += "clean" not in r.stdout
    assert crashes >= 1  # ratio 2 over up to 4 flushes a run: some run died mid-flush
    assert heights == sorted(heights)  # no stored block was lost across the crashes
    node, _ = node_factory((f"-datadir={d}",))
    c = client(node)
    h = c.getblockcount()
    assert h >= heights[-1]
    res = c.gettxoutsetinfo()
    assert res["hash_serialized_2"] == _expected_stats(c, h)[0]
    node.stop()
    node, _ = node_factory((f"-datadir={d}", "-reindex-chainstate"))
    c = client(node)
    assert node.state.rebuilt  # replayed from the stored blocks
    res2 = c.gettxoutsetinfo()
    assert c.getblockcount() == h
    for k in ("hash_serialized_2", "txouts", "transactions", "bogosize", "total_amount", "bestblock"):
        assert res2[k] == res[k], k


_CHILD_IDX = """
import sys
sys.path.insert(0, {root!r})
from nodexa_chain_core_amd.node import Node
from nodexa_chain_core_amd.utils.config import ArgsManager
from nodexa_chain_core_amd.rpc.client import RPCClient
a = ArgsManager()
a.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", "-datadir={d}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p", "-printtoconsole=0",
                    "-prune=1", "-addressindex", "-spentindex", "-dbcrashratio={ratio}"])
n = Node(a)
n.start()
c = RPCClient("127.0.0.1", n.rpc.port, "u", "p")
print("start", c.getblockcount(), n.state.rebuilt, flush=True)
for _ in range(3):
    c.generatetoaddress(2, {addr!r})
    c.gettxoutsetinfo()  # FlushStateToDisk: the crash points (indexes, then the coins)
n.stop()
print("clean", flush=True)
"""


def test_dbcrash_with_addressindex_on_pruned_node(core, node_factory, tmp_path):  # noqa: F811
    """a crash between the index write and the coins write of a flush leaves the indexes
    ahead of the chainstate. Start-up must rewind them (not replay from genesis, which a pruned node
    cannot do), and the address index must end with every coinbase exactly once."""
    d = tmp_path / "pruned"
    os.makedirs(d)
    node, addr = node_factory((f"-datadir={d}", "-prune=1", "-addressindex", "-spentindex"))
    node.state.store.set_max_file_size(4000)
    node.state.prune_after_height = 50
    c = client(node)
    c.generatetoaddress(400, addr)
    assert c.pruneblockchain(100) >= 100 and node.state.have_pruned
    node.stop()
    crashes, heights = 0, []
    for _ in range(5):
        r = subprocess.run([sys.executable, "-c", _CHILD_IDX.format(root=ROOT, d=d, ratio=2, addr=addr)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        starts = [x.split() for x in r.stdout.splitlines() if x.startswith("start")]
        assert len(starts) == 1 and starts[0][2] == "False", (r.stdout, r.stderr[-3000:])  # no genesis replay
        heights.append(int(starts[0][1]))
        crashes += "clean" not in r.stdout
    assert crashes >= 1 and heights == sorted(heights)
    log = open(os.path.join(d, "regtest", "debug.log")).read()
    assert "replaying from genesis" not in log and "Unable to rebuild" not in log
    assert "ahead of the UTXO set (interrupted flush); rewound" in log  # the crash point was hit and repaired
    node, _ = node_factory((f"-datadir={d}", "-prune=1", "-addressindex", "-spentindex"))
    c = client(node)
    h = c.getblockcount()
    utxos = c.getaddressutxos({"addresses": [addr]})
    assert sorted(u["height"] for u in utxos) == list(range(1, h + 1))  # each coinbase once, none lost
    bal = c.getaddressbalance({"addresses": [addr]})
    assert bal["balance"] == bal["received"] == sum(u["satoshis"] for u in utxos)
    node.stop()
