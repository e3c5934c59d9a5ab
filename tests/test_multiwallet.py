"""Several wallets in one node (-wallet=<file> given more than once) behind the /wallet/<name>
JSON-RPC endpoints (src/wallet/rpcwallet.cpp:40-78, wallet_multiwallet.py in the reference's
functional suite), the CLI's -rpcwallet and -stdinrpcpass."""
import io
import os

import pytest

from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures
from nodexa_chain_core_amd.rpc.client import RPCClient


def _wc(node, name):
    return RPCClient("127.0.0.1", node.rpc.port, "u", "p", wallet=name)


def test_multiwallet_endpoints(core, node_factory, tmp_path):  # noqa: F811
    node, _ = node_factory(("-wallet=wallet.json", "-wallet=w2.json"))
    c = client(node)
    assert c.listwallets() == ["wallet.json", "w2.json"]
    with pytest.raises(RuntimeError, match="RPC error -19"):
        c.getbalance()  # two wallets and the request names none
    with pytest.raises(RuntimeError, match="RPC error -18"):
        _wc(node, "nope.json").getbalance()
    w1, w2 = _wc(node, "wallet.json"), _wc(node, "w2.json")
    a2 = w2.getnewaddress()
    c.generatetoaddress(101, a2)  # not a wallet call: the plain endpoint serves it
    assert w2.getbalance() > 0 and w1.getbalance() == 0
    assert w2.validateaddress(a2)["ismine"] is True
    assert w1.validateaddress(a2)["ismine"] is False
    a1 = w1.getnewaddress()
    txid = w2.sendtoaddress(a1, 5)
    assert w1.getunconfirmedbalance() == 5 or w1.getbalance(None, 0) == 5
    assert any(t["txid"] == txid for t in w2.listtransactions("*", 50))
    assert os.path.exists(tmp_path / "regtest" / "w2.json") or os.path.exists(tmp_path / "w2.json")

    # the CLI picks the endpoint with -rpcwallet and can read the password from stdin
    from nodexa_chain_core_amd.rpc import client as cli

    base = ["-regtest", "-rpcuser=u", f"-rpcport={node.rpc.port}"]
    import sys

    old = sys.stdin
    try:
        sys.stdin = io.StringIO("p\n")
        assert cli.main(base + ["-stdinrpcpass", "-rpcwallet=w2.json", "getwalletinfo"]) == 0
        sys.stdin = io.StringIO("p\n")
        assert cli.main(base + ["-stdinrpcpass", "getwalletinfo"]) == 19  # RPC_WALLET_NOT_SPECIFIED
    finally:
        sys.stdin = old


def test_multiwallet_restart_and_bad_names(core, node_factory, tmp_path):  # noqa: F811
    node, _ = node_factory(("-wallet=wallet.json", "-wallet=w2.json"))
    a2 = _wc(node, "w2.json").getnewaddress()
    node.stop()
    node, _ = node_factory(("-wallet=wallet.json", "-wallet=w2.json"))
    assert _wc(node, "w2.json").validateaddress(a2)["ismine"] is True  # keys reloaded from w2.json
    node.stop()
    single, _ = node_factory(("-wallet=w2.json",))
    assert client(single).validateaddress(a2)["ismine"] is True  # one wallet: the plain endpoint is it
    single.stop()
    with pytest.raises(SystemExit, match="not a path"):
        node_factory(("-wallet=../w3.json",))
    with pytest.raises(SystemExit, match="Duplicate"):
        node_factory(("-wallet=w2.json", "-wallet=w2.json"))
