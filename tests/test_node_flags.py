"""Operator flags of the reference daemon that shape the RPC server, notifications, logging and
the process (src/init.cpp, src/httpserver.cpp, src/httprpc.cpp):

* -rpcauth=<user>:<salt>$<hmac-sha256(salt, password)> (share/rpcauth; multiUserAuthorized),
  -rpcallowip (ClientAllowed: loopback always, others by address or subnet, 403 otherwise),
  -rpcthreads (workers executing requests), -rpcservertimeout, -rpccookiefile, -rest (off by
  default, as DEFAULT_REST_ENABLE);
* -blocknotify / -walletnotify with "%s" substitution;
* -logtimestamps / -logtimemicros, -shrinkdebugfile, -pid.
"""
import base64
import hashlib
import hmac
import http.client
import json
import os
import time

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from wallet_util import fund


def _post(port, user, pw, method="getblockcount"):
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    tok = base64.b64encode(f"{user}:{pw}".encode()).decode()
    conn.request("POST", "/", json.dumps({"id": 1, "method": method, "params": []}),
                 {"Authorization": "Basic " + tok, "Content-Type": "application/json"})
    r = conn.getresponse()
    body = r.read()
    conn.close()
    return r.status, body


def _wait_for(pred, timeout=10.0):
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return True
        time.sleep(0.05)
    return False


def test_rpcauth_allowip_and_rest_default(core, node_factory):  # noqa: F811
    salt = "cb77f0957de88ff388cf817ddbc7273"
    digest = hmac.new(salt.encode(), b"hunter2", hashlib.sha256).hexdigest()
    node, _ = node_factory((f"-rpcauth=alice:{salt}${digest}", "-rpcallowip=10.0.0.0/8", "-rpcthreads=2",
                            "-norest"))
    port = node.rpc.port
    assert _post(port, "alice", "hunter2")[0] == 200
    assert _post(port, "alice", "wrong")[0] == 401
    assert _post(port, "u", "p")[0] == 200  # -rpcuser / -rpcpassword still work next to -rpcauth
    srv = node.rpc.httpd
    assert srv.client_allowed("127.0.0.1") and srv.client_allowed("::1")
    assert srv.client_allowed("10.1.2.3") and not srv.client_allowed("192.168.1.1")
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    conn.request("GET", "/rest/chaininfo.json")
    assert conn.getresponse().status == 404  # REST is opt-in (-rest)
    conn.close()


def test_rpc_allowip_subnet_forms():
    from nodexa_chain_core_amd.rpc.server import parse_allow_subnets

    nets = parse_allow_subnets(["192.168.0.0/255.255.0.0", "172.16.5.4", "fd00::/8"])
    from nodexa_chain_core_amd.rpc.server import ip_allowed

    assert ip_allowed("192.168.7.9", nets) and ip_allowed("172.16.5.4", nets) and ip_allowed("fd00::1", nets)
    assert not ip_allowed("172.16.5.5", nets) and not ip_allowed("8.8.8.8", nets)
    with pytest.raises(ValueError):
        parse_allow_subnets(["not-an-ip"])


def test_notifications_and_logging(core, node_factory, tmp_path):  # noqa: F811
    blk = tmp_path / "blocks.txt"
    wtx = tmp_path / "wallet.txt"
    node, addr = node_factory((f"-blocknotify=echo %s >> {blk}", f"-walletnotify=echo %s >> {wtx}",
                               "-logtimemicros", "-pid=nodexa_test.pid", "-rest"))
    c = client(node)
    h = c.generatetoaddress(2, addr)
    assert _wait_for(lambda: blk.exists() and len(blk.read_text().split()) >= 2)
    assert set(blk.read_text().split()) >= set(h)
    w = fund(c, 101)
    txid = c.sendtoaddress(w, 1.0)
    assert _wait_for(lambda: wtx.exists() and txid in wtx.read_text().split())
    pidfile = os.path.join(node.datadir, "nodexa_test.pid")
    assert open(pidfile).read().strip() == str(os.getpid())
    from nodexa_chain_core_amd.utils import log

    assert log.timestamp_format(1_700_000_000.123456).endswith(".123456Z")
    conn = http.client.HTTPConnection("127.0.0.1", node.rpc.port, timeout=5)
    conn.request("GET", "/rest/chaininfo.json")
    assert conn.getresponse().status == 200
    conn.close()
    node.stop()
    assert not os.path.exists(pidfile)


def test_shrink_debug_file(tmp_path):
    from nodexa_chain_core_amd.utils import log

    p = tmp_path / "debug.log"
    p.write_bytes(b"x" * (12 * 1_000_000) + b"\nlast line\n")
    log.shrink_debug_file(str(p))
    data = p.read_bytes()
    assert len(data) <= 10 * 1_000_000 + 16 and data.endswith(b"last line\n")
    small = tmp_path / "small.log"
    small.write_bytes(b"keep\n")
    log.shrink_debug_file(str(small))
    assert small.read_bytes() == b"keep\n"


def test_relay_package_and_block_policy_flags(core, node_factory):  # noqa: F811
    """-datacarrier, -limitancestorcount, -maxtxfee, -blockmintxfee and -mempoolexpiry."""
    from wallet_util import spend

    node, addr = node_factory(("-acceptnonstdtxn=0", "-datacarrier=0", "-limitancestorcount=2", "-maxtxfee=0.5",
                               "-blockmintxfee=0.05", "-mempoolexpiry=1"))
    c = client(node)
    w = fund(c, 110)
    coins = sorted((u for u in c.listunspent() if u["spendable"]), key=lambda u: u["txid"])
    # -datacarrier=0: an OP_RETURN output is non-standard
    u = coins.pop()
    raw = c.createrawtransaction([{"txid": u["txid"], "vout": u["vout"]}], {"data": "00" * 8, w: 1.0})
    signed = c.signrawtransaction(raw)["hex"]
    assert c.testmempoolaccept([signed])[0]["reject-reason"].endswith("scriptpubkey")
    # -maxtxfee=0.5: a 1 CLORE fee is absurd unless allowhighfees
    u = coins.pop()
    hi = spend(c, u["txid"], u["vout"], u["amount"], w, 1.0, fee=1.0)
    with pytest.raises(RuntimeError, match="absurdly-high-fee"):
        c.sendrawtransaction(hi)
    assert c.sendrawtransaction(hi, True)
    # -limitancestorcount=2: a third unconfirmed generation is refused
    u = coins.pop()
    t1 = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], w, 5.0))
    t2 = c.sendrawtransaction(spend(c, t1, 0, 5.0, w, 4.0))
    t3 = spend(c, t2, 0, 4.0, w, 3.0)
    with pytest.raises(RuntimeError, match="too-long-mempool-chain"):
        c.sendrawtransaction(t3)
    # -blockmintxfee=0.05 CLORE/kB: the 0.01-fee transactions (~4.4M sat/kB) stay out of templates
    # while the 1 CLORE one (above the floor) goes in
    tpl = {t["txid"] for t in c.getblocktemplate({"rules": ["segwit"]})["transactions"]}
    assert t1 not in tpl and t2 not in tpl and c.decoderawtransaction(hi)["txid"] in tpl
    # -mempoolexpiry=1 (hour): two hours later the next admission expires the old entries
    pool_before = set(c.getrawmempool())
    assert {t1, t2} <= pool_before
    c.setmocktime(int(time.time()) + 2 * 3600)
    u = coins.pop()
    fresh = c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], w, 1.0))
    assert set(c.getrawmempool()) == {fresh}
    c.setmocktime(0)


def test_wallet_flags(core, node_factory, tmp_path):  # noqa: F811
    """-keypool, -mintxfee, -maxtxfee (wallet cap) and -walletbroadcast=0."""
    node, addr = node_factory(("-keypool=5", "-mintxfee=0.05", "-walletbroadcast=0"))
    c = client(node)
    assert len(node.wallet.pool) >= 5 or node.wallet.keypool_size == 5
    w = fund(c, 101)
    txid = c.sendtoaddress(w, 1.0)
    assert txid not in c.getrawmempool()  # recorded in the wallet, not broadcast
    t = c.gettransaction(txid)
    size = len(bytes.fromhex(t["hex"]))
    assert -t["fee"] * 1e8 * 1000 / size >= 5_000_000 * 0.99  # -mintxfee floor (sat per kB)
    node.stop()
    os.makedirs(tmp_path / "n2", exist_ok=True)
    node2, _ = node_factory((f"-datadir={tmp_path / 'n2'}", "-maxtxfee=0.0001"))
    c2 = client(node2)
    w2 = fund(c2, 101)
    with pytest.raises(RuntimeError, match="maxtxfee"):
        c2.sendtoaddress(w2, 1.0)


def test_p2p_flags(core, node_factory, tmp_path):  # noqa: F811
    """-uacomment, -whitelist, -blocksonly, -peerbloomfilters=0 and -externalip."""
    a, addr = node_factory(("-listen=1", "-port=0", "-listenonion=0", "-uacomment=gpu-node", "-whitelist=127.0.0.1",
                            "-blocksonly", "-peerbloomfilters=0", "-externalip=203.0.113.7"))
    client(a).generatetoaddress(2, addr)
    os.makedirs(tmp_path / "b", exist_ok=True)
    b, _ = node_factory((f"-datadir={tmp_path / 'b'}", f"-connect=127.0.0.1:{a.connman.port}"))
    cb = client(b)
    assert _wait_for(lambda: cb.getblockcount() == 2, 20)
    peer_a = cb.getpeerinfo()[0]
    assert peer_a["subver"].endswith("(gpu-node)/")
    assert int(peer_a["services"], 16) & (1 << 2) == 0  # NODE_BLOOM off
    assert peer_a["relaytxes"] is False                  # -blocksonly announces relay=false
    ca = client(a)
    assert _wait_for(lambda: ca.getpeerinfo() and ca.getpeerinfo()[0]["whitelisted"] is True)
    local = {(x["address"], x["port"]) for x in ca.getnetworkinfo()["localaddresses"]}
    assert ("203.0.113.7", a.connman.port) in local
    # a bloom filter message to a node without NODE_BLOOM costs the peer 100 points, but a
    # whitelisted peer is never banned
    peer_b = a.connman.peers[0]
    a.connman.on_filterload(peer_b, b"\x01\x00" + bytes(9))
    assert peer_b.misbehavior >= 100 and not a.connman.is_banned("127.0.0.1")


def test_whitebind_and_socket_buffers(core, node_factory, tmp_path):  # noqa: F811
    """-whitebind: peers accepted on that socket are whitelisted whatever their address (and a
    banned address still gets in there); -bind / -listen keep the ordinary socket; -maxsendbuffer /
    -maxreceivebuffer size each peer's socket buffers."""
    import socket

    a, addr = node_factory(("-listen=1", "-bind=127.0.0.1:0", "-whitebind=127.0.0.1:0", "-listenonion=0",
                            "-maxsendbuffer=200", "-maxreceivebuffer=300"))
    cm = a.connman
    white_port = cm._extra_servers[0].getsockname()[1]
    assert cm.port and white_port != cm.port
    client(a).generatetoaddress(2, addr)
    cm.ban("127.0.0.1", 3600)
    os.makedirs(tmp_path / "b", exist_ok=True)
    b, _ = node_factory((f"-datadir={tmp_path / 'b'}", f"-connect=127.0.0.1:{white_port}"))
    assert _wait_for(lambda: client(b).getblockcount() == 2, 20)
    ca = client(a)
    assert _wait_for(lambda: ca.getpeerinfo() and ca.getpeerinfo()[0]["whitelisted"] is True)
    sock = cm.peers[0].sock
    # Linux doubles the requested size for its bookkeeping (and caps it at wmem_max / rmem_max)
    assert 2 * 4096 <= sock.getsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF) <= 2 * 200_000
    assert 2 * 4096 <= sock.getsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF) <= 2 * 300_000


def test_cli_stdin_and_rpcwait(core, node_factory, tmp_path, capsys, monkeypatch):  # noqa: F811
    import io

    from nodexa_chain_core_amd.rpc import client as cli

    node, addr = node_factory()
    port = node.rpc.port
    base = ["-regtest", "-rpcuser=u", "-rpcpassword=p", f"-rpcport={port}"]
    monkeypatch.setattr("sys.stdin", io.StringIO("1\n"))
    assert cli.main(base + ["-stdin", "getblockhash"]) == 8  # abs(RPC_INVALID_PARAMETER): no height 1 yet
    client(node).generatetoaddress(1, addr)
    monkeypatch.setattr("sys.stdin", io.StringIO("1\n"))
    capsys.readouterr()
    assert cli.main(base + ["-stdin", "getblockhash"]) == 0
    assert len(capsys.readouterr().out.strip()) == 64
    # nothing listens on this port: without -rpcwait the CLI fails at once
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    dead = s.getsockname()[1]
    s.close()
    assert cli.main(["-regtest", "-rpcuser=u", "-rpcpassword=p", f"-rpcport={dead}", "getblockcount"]) != 0


def test_chain_flags_loadblock_assumevalid_vbparams_checkblocks(core, node_factory, tmp_path):  # noqa: F811
    """-loadblock (+ -stopafterblockimport), -assumevalid, -vbparams, -checkblocks/-checklevel and
    getblockchaininfo.initialblockdownload."""
    src, addr = node_factory((f"-datadir={tmp_path / 'src'}",) if os.makedirs(tmp_path / "src") is None else ())
    c = client(src)
    hashes = c.generatetoaddress(12, addr)
    assert c.getblockchaininfo()["initialblockdownload"] is False
    headers = [src.state.get_block(bytes.fromhex(h)[::-1]).header for h in hashes]
    src.stop()
    blk0 = os.path.join(src.datadir, "blocks", "blk00000.dat")
    # import the first node's block file into a fresh node, with every script check skipped up to
    # the assumed-valid tip
    os.makedirs(tmp_path / "dst")
    dst, _ = node_factory((f"-datadir={tmp_path / 'dst'}", f"-loadblock={blk0}", f"-assumevalid={hashes[-1]}",
                           "-vbparams=testdummy:0:1", "-checkblocks=12", "-checklevel=3"))
    cd = client(dst)
    assert cd.getblockcount() == 12 and cd.getbestblockhash() == hashes[-1]
    # blocks read one by one: the assumed-valid header is known only when its own block arrives,
    # so only that block skips its scripts (as LoadExternalBlockFile in the reference)
    assert dst.state.scripts_skipped == 1
    td = {d.name: d for d in dst.state.versionbits.deployments}["testdummy"]
    assert (td.start, td.timeout) == (0, 1)
    dst.stop()
    # restart with start-up block verification over the imported chain
    dst2, _ = node_factory((f"-datadir={tmp_path / 'dst'}", "-checkblocks=12", "-checklevel=2"))
    assert client(dst2).getblockcount() == 12
    dst2.stop()
    # headers first (as P2P sync delivers them): every ancestor of the assumed-valid block skips
    os.makedirs(tmp_path / "hf")
    hf, _ = node_factory((f"-datadir={tmp_path / 'hf'}", f"-assumevalid={hashes[-1]}"))
    res = hf.state.chain.accept_headers(headers, int(time.time()) + 7200, True)
    assert all(r.ok for r in res)
    assert hf.state.load_external_block_file(blk0) == 12 and hf.state.scripts_skipped == 12
    hf.stop()
    with pytest.raises(SystemExit, match="regtest|malformed|Invalid deployment"):
        node_factory((f"-datadir={tmp_path / 'dst'}", "-vbparams=nosuch:0:1"))


def test_dbcrashratio_crash_and_recovery(core, node_factory, tmp_path):  # noqa: F811
    """-dbcrashratio=1 kills the daemon in the middle of its flush
    (feature_dbcrash.py); the next start notices the mismatch and replays the blocks."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = tmp_path / "crash"
    os.makedirs(d)
    code = f"""
import sys
sys.path.insert(0, {root!r})
from nodexa_chain_core_amd.node import Node
from nodexa_chain_core_amd.utils.config import ArgsManager
from nodexa_chain_core_amd import _core
a = ArgsManager()
a.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", "-datadir={d}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p", "-printtoconsole=0",
                    "-dbcrashratio=1"])
n = Node(a)
n.start()
addr = _core.base58check_encode(bytes([42]) + bytes(range(20)))
from nodexa_chain_core_amd.rpc.client import RPCClient
RPCClient("127.0.0.1", n.rpc.port, "u", "p").generatetoaddress(5, addr)
n.stop()
print("not reached")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "not reached" not in r.stdout, r.stderr[-2000:]
    # (LevelDB layout: the crash comes before the flush's one atomic batch of coins + assets)
    assert os.path.exists(d / "regtest" / "chainstate" / "CURRENT") or os.path.exists(d / "chainstate" / "CURRENT")
    node, _ = node_factory((f"-datadir={d}",))
    assert client(node).getblockcount() == 5
    assert client(node).gettxoutsetinfo()["height"] == 5


class _FakePeer:
    def __init__(self, pid=99):
        self.id, self.addr, self.sent = pid, ("127.0.0.1", 1), []
        self.known_txs, self.whitelisted, self.misbehavior = set(), False, 0

    def send(self, cmd, payload=b""):
        self.sent.append((cmd, payload))

    def misbehaving(self, score, why):
        self.misbehavior += score


def test_orphan_transactions_and_maxorphantx(core, node_factory):  # noqa: F811
    """A child that arrives before its parent waits in the orphan pool, the parent is requested
    with getdata, and both enter the mempool once the parent arrives (net_processing's orphan
    handling); -maxorphantx bounds the pool and a disconnect erases the peer's orphans."""
    from wallet_util import spend

    node, addr = node_factory(("-listen=1", "-port=0", "-listenonion=0", "-maxorphantx=3"))
    c = client(node)
    w = fund(c, 105)
    coins = sorted((u for u in c.listunspent() if u["spendable"]), key=lambda u: u["txid"])
    cm = node.connman
    assert cm.max_orphans == 3
    u = coins.pop()
    parent_hex = spend(c, u["txid"], u["vout"], u["amount"], w, 5.0)
    parent = core.Transaction.deserialize(bytes.fromhex(parent_hex))
    ptxid = parent.txid()[::-1].hex()
    raw = c.createrawtransaction([{"txid": ptxid, "vout": 0}], {w: 4.99})
    prev = [{"txid": ptxid, "vout": 0, "scriptPubKey": parent.vout[0].script_pubkey.hex(), "amount": 5.0}]
    signed = c.signrawtransaction(raw, prev)
    assert signed["complete"], signed
    child = core.Transaction.deserialize(bytes.fromhex(signed["hex"]))
    peer = _FakePeer()
    cm.on_tx(peer, child.serialize(True))
    assert child.txid() in cm.orphans and child.txid() not in node.state.mempool
    assert peer.sent and peer.sent[-1][0] == "getdata" and parent.txid() in peer.sent[-1][1]
    cm.on_tx(peer, parent.serialize(True))
    assert parent.txid() in node.state.mempool and child.txid() in node.state.mempool
    assert not cm.orphans
    # the pool is capped at -maxorphantx; a disconnect removes what that peer sent
    for k in range(5):
        fake = core.Transaction.deserialize(bytes.fromhex(
            c.createrawtransaction([{"txid": "%064x" % (k + 1), "vout": 0}], {w: 0.5})))
        cm.on_tx(peer, fake.serialize(True))
    assert len(cm.orphans) == 3
    cm.erase_orphans_for(peer.id)
    assert not cm.orphans and not cm.orphans_by_prev


def test_maxmempool_trim_and_rolling_min_fee(core, node_factory):  # noqa: F811
    """TrimToSize: over the limit the lowest-feerate package leaves and the pool's minimum fee
    rises to its feerate plus the incremental relay fee; getmempoolinfo reports both; the floor
    decays once a block arrives. (-maxmempool below 10 MB is refused as in the reference, so the
    limit is lowered on the state object to keep the test small.)"""
    from wallet_util import spend

    node, addr = node_factory()
    c = client(node)
    w = fund(c, 110)
    st = node.state
    coins = sorted((u for u in c.listunspent() if u["spendable"]), key=lambda u: u["txid"])
    fees = [0.02, 0.03, 0.05, 0.01]
    ids = []
    for f in fees[:3]:
        u = coins.pop()
        ids.append(c.sendrawtransaction(spend(c, u["txid"], u["vout"], u["amount"], w, 1.0, fee=f)))
    st.max_mempool_bytes = st.mempool_usage() - 1  # one entry too many
    assert st.trim_mempool() == 1
    pool = set(c.getrawmempool())
    assert ids[0] not in pool and ids[1] in pool and ids[2] in pool  # the 0.02-fee tx went
    info = c.getmempoolinfo()
    assert info["maxmempool"] == st.max_mempool_bytes and info["mempoolminfee"] > info["minrelaytxfee"]
    floor = st.mempool_min_fee()
    assert floor > st.incremental_relay_fee
    u = coins.pop()  # below the new floor: refused
    cheap = spend(c, u["txid"], u["vout"], u["amount"], w, 1.0, fee=fees[3])
    with pytest.raises(RuntimeError, match="mempool min fee not met"):
        c.sendrawtransaction(cheap)
    # a block resets the decay clock; a week later (3 h half-life while nearly empty) it is gone
    st.max_mempool_bytes = 300_000_000
    c.generatetoaddress(1, addr)
    c.setmocktime(int(time.time()) + 7 * 24 * 3600)
    assert st.mempool_min_fee() == 0
    c.setmocktime(0)
    node.stop()
    with pytest.raises(SystemExit, match="maxmempool must be at least"):
        node_factory(("-maxmempool=5",))


def test_timedata_median_and_limit():
    from nodexa_chain_core_amd.net.timedata import TimeData

    td = TimeData(max_adjustment=600)
    offsets = [30, 40, 50, 60]
    for i, o in enumerate(offsets):
        td.add(f"10.0.0.{i}", o)
    assert td.offset == 40  # 5 samples with our own 0: median of [0, 30, 40, 50, 60]
    td.add("10.0.0.1", 9999)  # one sample per address
    assert td.offset == 40
    far = TimeData(max_adjustment=600)
    for i in range(6):
        far.add(f"10.1.0.{i}", 3600)
    assert far.offset == 0  # median beyond -maxtimeadjustment: no adjustment


def test_dns_seeding(core, node_factory):  # noqa: F811
    node, _ = node_factory(("-listen=1", "-port=0", "-listenonion=0", "-maxconnections=0"))
    cm = node.connman
    cm.dns_seeds = ["seed.example"]
    calls = []

    def fake_resolve(host, port, *a):
        calls.append((host, port))
        return [(2, 1, 6, "", ("198.51.100.7", port)), (2, 1, 6, "", ("198.51.100.8", port))]
    assert cm.dns_address_seed(fake_resolve) == 2
    assert calls == [("seed.example", node.params.default_port)] and cm.addrman.size() == 2
    assert cm.dns_address_seed(fake_resolve) == 0  # addrman has peers now: skipped
    cm.force_dns_seed = True
    assert cm.dns_address_seed(lambda *a: (_ for _ in ()).throw(OSError("offline"))) == 0


def test_zapwallettxes_and_rescan(core, node_factory, tmp_path):  # noqa: F811
    d = tmp_path / "zap"
    os.makedirs(d)
    node, _ = node_factory((f"-datadir={d}",))
    c = client(node)
    w = fund(c, 101)
    txid = c.sendtoaddress(w, 1.0, "rent", "bob")
    c.generatetoaddress(1, w)
    before = {t["txid"] for t in c.listtransactions("*", 1000)}
    node.stop()
    node2, _ = node_factory((f"-datadir={d}", "-zapwallettxes=1"))
    c2 = client(node2)
    after = {t["txid"] for t in c2.listtransactions("*", 1000)}
    assert after == before  # everything confirmed comes back from the rescan
    assert c2.gettransaction(txid).get("comment") == "rent"  # mode 1 keeps the metadata
    node2.stop()
    node3, _ = node_factory((f"-datadir={d}", "-zapwallettxes=2"))
    assert "comment" not in client(node3).gettransaction(txid) or not client(node3).gettransaction(txid)["comment"]
    node3.stop()
    node4, _ = node_factory((f"-datadir={d}", "-rescan"))
    assert {t["txid"] for t in client(node4).listtransactions("*", 1000)} == before


def test_checkpoints_mocktime_discover(core, node_factory, tmp_path):  # noqa: F811
    main = core.make_chain_params("main")
    assert main.checkpoints
    main.clear_checkpoints()
    assert not main.checkpoints
    node, _ = node_factory(("-mocktime=1700000000", "-listen=1", "-port=0", "-listenonion=0"))
    assert node.state.adjusted_time() == 1700000000
    cm = node.connman
    n = cm.discover_local_addresses(lambda: [(2, 1, 6, "", ("10.0.0.5", 0)), (2, 1, 6, "", ("8.8.4.4", 0)),
                                             (2, 1, 6, "", ("127.0.0.1", 0))])
    assert n == 1 and ("8.8.4.4", cm.port) in cm.local_addrs


def test_maxuploadtarget(core, node_factory):  # noqa: F811
    node, _ = node_factory(("-listen=1", "-port=0", "-listenonion=0", "-maxuploadtarget=200"))
    cm = node.connman
    info = client(node).getnettotals()["uploadtarget"]
    assert info["target"] == 200 * 1024 * 1024 and info["serve_historical_blocks"] is False  # < one day of blocks
    assert info["target_reached"] is False
    cm.max_outbound_limit = 2_000_000_000
    cm.record_sent(10)
    assert cm.upload_target_info()["serve_historical_blocks"] is True
    cm.record_sent(2_000_000_000)
    t = cm.upload_target_info()
    assert t["target_reached"] and not t["serve_historical_blocks"] and t["bytes_left_in_cycle"] == 0


def test_spend_zeroconf_change_and_rpcserialversion(core, node_factory, tmp_path):  # noqa: F811
    node, addr = node_factory(("-rpcserialversion=0",))
    c = client(node)
    w = fund(c, 101)  # exactly one mature coinbase
    coin = [u for u in c.listunspent() if u["spendable"]][0]["amount"]
    t1 = c.sendtoaddress(addr, round(coin / 2, 8))  # the change stays unconfirmed
    t2 = c.sendtoaddress(addr, round(coin / 4, 8))  # only possible by spending that change
    pool = c.getrawmempool()
    assert t1 in pool and t2 in pool
    raw = c.getrawtransaction(t2)
    assert core.Transaction.deserialize(bytes.fromhex(raw)).serialize(False).hex() == raw  # no witness form
    node.stop()
    os.makedirs(tmp_path / "nz")
    node2, addr2 = node_factory((f"-datadir={tmp_path / 'nz'}", "-spendzeroconfchange=0"))
    c2 = client(node2)
    fund(c2, 101)
    coin2 = [u for u in c2.listunspent() if u["spendable"]][0]["amount"]
    c2.sendtoaddress(addr2, round(coin2 / 2, 8))
    with pytest.raises(RuntimeError, match="Insufficient funds"):
        c2.sendtoaddress(addr2, round(coin2 / 4, 8))


def test_removed_flags(core, node_factory, tmp_path):  # noqa: F811
    for i, bad in enumerate(("-socks=4", "-rpcssl=1", "-tor=127.0.0.1:9050")):
        d = tmp_path / f"old{i}"
        os.makedirs(d)
        with pytest.raises(SystemExit, match="socks|SSL|onion"):
            node_factory((f"-datadir={d}", bad))
    node, _ = node_factory(("-benchmark", "-debugnet"))  # accepted with a warning
    assert client(node).getblockcount() == 0


def test_checkblockindex(core, node_factory):  # noqa: F811
    node, addr = node_factory(("-checkblockindex",))
    c = client(node)
    c.generatetoaddress(15, addr)
    tip = c.getbestblockhash()
    c.invalidateblock(c.getblockhash(10))  # disconnect back to height 9
    node.state.check_block_index()
    assert c.getblockcount() == 9
    c.reconsiderblock(tip)
    node.state.check_block_index()
    assert c.getbestblockhash() == tip
    c.generatetoaddress(3, addr)  # the checker runs inside every ProcessNewBlock
    assert c.getblockcount() == 18
