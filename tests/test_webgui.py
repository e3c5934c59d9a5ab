"""The web wallet (gui/index.html; the reference's Qt GUI role, src/qt/): served at /gui behind the
RPC credentials, every RPC the page calls is registered, and the fields each page reads are in
those RPCs' replies (the page is static, so this pins its contract with the node)."""
import base64
import http.client
import json
import os
import re
import shutil
import subprocess

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures


def _get(port, path, auth=None):
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    headers = {"Authorization": "Basic " + base64.b64encode(auth.encode()).decode()} if auth else {}
    conn.request("GET", path, headers=headers)
    r = conn.getresponse()
    body = r.read()
    conn.close()
    return r.status, r.getheader("Content-Type"), body


def test_gui_served_behind_auth_and_its_rpc_contract(core, node_factory):  # noqa: F811
    node, addr = node_factory(("-webgui",))
    port = node.rpc.port
    assert _get(port, "/gui")[0] == 401
    assert _get(port, "/gui", "u:wrong")[0] == 401
    status, ctype, body = _get(port, "/gui", "u:p")
    assert status == 200 and ctype.startswith("text/html")
    page = body.decode()
    assert "<title>Nodexa wallet</title>" in page
    methods = set(re.findall(r'rpc\("(\w+)"', page))
    assert {"getwalletinfo", "sendtoaddress", "getnewaddress", "listtransactions", "listmyassets", "transfer", "issue",
            "setgenerate", "getpeerinfo"} <= methods
    assert methods <= set(node.table.commands), methods - set(node.table.commands)

    c = client(node)
    c.generatetoaddress(101, c.getnewaddress())
    w = c.getwalletinfo()
    assert {"balance", "unconfirmed_balance", "immature_balance"} <= set(w) and w["balance"] > 0
    ch = c.getblockchaininfo()
    assert {"blocks", "chain", "initialblockdownload"} <= set(ch)
    assert {"connections", "subversion"} <= set(c.getnetworkinfo())
    txs = c.listtransactions("*", 10)
    assert txs and {"time", "category", "amount", "confirmations", "txid"} <= set(txs[0])
    recv = c.listreceivedbyaddress(0, True)
    assert recv and {"address", "amount", "confirmations"} <= set(recv[0])
    assert isinstance(c.listmyassets(), dict)
    m = c.getmininginfo()
    assert {"hashespersec", "networkhashps", "difficulty", "blocks", "pooledtx"} <= set(m)
    assert c.getgenerate() in (True, False)
    try:  # (the peers page shows the error instead when P2P is off, as the reference's RPC raises it)
        assert {"totalbytesrecv", "totalbytessent"} <= set(c.getnettotals())
    except RuntimeError as e:
        assert "Peer-to-peer functionality missing or disabled" in str(e)
    assert c.validateaddress(addr)["isvalid"]
    # the send flow of the page
    dest = c.getnewaddress("gui")
    txid = c.sendtoaddress(dest, 1.5, "from the gui", "", False)
    assert txid in c.getrawmempool()


@pytest.mark.skipif(shutil.which("node") is None, reason="no Node.js to run the page's script")
def test_gui_script_drives_the_node(core, node_factory):  # noqa: F811
    """The page's own JavaScript, run under Node.js with a DOM stub against the live node: the
    overview shows the balance, a new receiving address, a payment sent from the send page, the
    transactions / mining / peers pages and the RPC console."""
    node, _ = node_factory(("-webgui",))
    c = client(node)
    c.generatetoaddress(101, c.getnewaddress())
    dest = c.getnewaddress("dest")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    page = os.path.join(root, "nodexa_chain_core_amd", "gui", "index.html")
    r = subprocess.run(["node", os.path.join(root, "tests", "gui_harness.js"), page, str(node.rpc.port), "u:p", dest],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert float(out["available"]) > 0 and out["blocks"].startswith("101")
    assert "regtest" in out["status"] and out["recentRows"] > 0
    assert out["receiveClass"].endswith("ok") and c.validateaddress(out["newAddress"])["isvalid"]
    assert out["send"].startswith("sent: ")
    txid = out["send"].split()[-1]
    assert txid in c.getrawmempool() and c.gettransaction(txid)["amount"] == 0  # to our own address
    assert out["txRows"] > 0 and out["mining"]
    assert "getblockcount" in out["console"] and c.getblockhash(1) in out["console"]
    assert out["activeSection"] == ["peers"]


def test_gui_can_be_disabled(core, node_factory):  # noqa: F811
    node, _ = node_factory(("-webgui=0",))
    assert _get(node.rpc.port, "/gui", "u:p")[0] == 405
    node.stop()
    node2, _ = node_factory()  # off by default
    assert _get(node2.rpc.port, "/gui", "u:p")[0] == 405


def _post(port, body: bytes, headers: dict):
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    h = {"Authorization": "Basic " + base64.b64encode(b"u:p").decode()}
    h.update(headers)
    conn.request("POST", "/", body=body, headers=h)
    r = conn.getresponse()
    out = r.read()
    conn.close()
    return r.status, out


def test_cross_site_posts_are_refused(core, node_factory):  # noqa: F811
    """with the browser holding the RPC credentials, a cross-site form POST
    (text/plain body that parses as JSON-RPC) must not run; the served page's own requests must."""
    node, _ = node_factory(("-webgui",))
    port = node.rpc.port
    body = b'{"method": "getblockcount", "params": [], "id": 1}'
    evil = {"Content-Type": "text/plain", "Origin": "http://evil.example", "Sec-Fetch-Site": "cross-site"}
    assert _post(port, body, evil)[0] == 403
    same_origin_no_token = {"Origin": f"http://127.0.0.1:{port}", "Content-Type": "application/json"}
    assert _post(port, body, same_origin_no_token)[0] == 403
    assert _post(port, body, {"Referer": "http://evil.example/x", "X-Nodexa-CSRF": "guess"})[0] == 403
    page = _get(port, "/gui", "u:p")[2].decode()
    token = re.search(r'const CSRF = "([0-9a-f]{32})"', page).group(1)
    ok = {"Origin": f"http://127.0.0.1:{port}", "X-Nodexa-CSRF": token, "Content-Type": "application/json"}
    status, out = _post(port, body, ok)
    assert status == 200 and json.loads(out)["result"] == 0
    assert _post(port, body, dict(ok, Origin="http://evil.example"))[0] == 403  # the token alone is not enough
    status, out = _post(port, body, {"Content-Type": "text/plain"})  # curl / nodexa-cli: no browser headers
    assert status == 200 and json.loads(out)["result"] == 0
