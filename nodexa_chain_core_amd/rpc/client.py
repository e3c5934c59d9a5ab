"""JSON-RPC client and the `nodexa-cli` command line.

Parity: clore-cli CallRPC / CommandLineRPC (src/clore-cli.cpp:288-381): HTTP
POST with Basic auth (rpcuser/rpcpassword or the data-dir cookie), positional
string arguments converted to JSON for the parameters listed in the
reference's conversion table (src/rpc/client.cpp: vRPCConvertParams), `-named`
arguments, result printed as JSON (strings raw), exit code = error code.
"""
from __future__ import annotations

import base64
import http.client
import json
import os
import sys
import time
import urllib.parse

from ..utils.config import ArgsManager

# params parsed as JSON when given as CLI strings, by method and position: the reference's
# vRPCConvertParams (src/rpc/client.cpp), plus this engine's verifyheaders
_CONVERT_POSITIONS = {
    "issue": (1, 4, 5, 6), "issuerestrictedasset": (1, 5, 6, 7), "issuequalifierasset": (1, 4),
    "reissuerestrictedasset": (1, 3, 6, 7), "issueunique": (1, 2), "transfer": (1, 4), "transferfromaddress":
    (2, 5), "transferfromaddresses": (1, 2, 5), "transferqualifier": (2, 5), "reissue": (1, 4, 5),
    "listmyassets": (1, 2, 3, 4), "listassets": (1, 2, 3), "setmocktime": (0,), "generate": (0, 1),
    "setgenerate": (0, 1), "generatetoaddress": (0, 2), "getnetworkhashps": (0, 1), "sendtoaddress": (1, 4),
    "sendfromaddress": (2, 5), "settxfee": (0,), "getreceivedbyaddress": (1,), "getreceivedbyaccount": (1,),
    "listreceivedbyaddress": (0, 1, 2), "listreceivedbyaccount": (0, 1, 2), "getbalance": (1, 2),
    "getblockhash": (0,), "waitforblockheight": (0, 1), "waitforblock": (1,), "waitfornewblock": (0,), "move":
    (2, 3), "sendfrom": (2, 3), "listtransactions": (1, 2, 3), "listaccounts": (0, 1), "walletpassphrase": (1,),
    "getblocktemplate": (0,), "listsinceblock": (1, 2, 3), "sendmany": (1, 2, 4), "addmultisigaddress": (0, 1),
    "createmultisig": (0, 1), "listunspent": (0, 1, 2, 3, 4), "getblock": (1,), "getblockheader": (1,),
    "getchaintxstats": (0,), "gettransaction": (1,), "getrawtransaction": (1,), "createrawtransaction": (0, 1,
    2, 3), "signrawtransaction": (1, 2), "sendrawtransaction": (1,), "testmempoolaccept": (0, 1),
    "combinerawtransaction": (0,), "fundrawtransaction": (1,), "gettxout": (1, 2), "gettxoutproof": (0,),
    "lockunspent": (0, 1), "importprivkey": (2,), "importaddress": (2, 3), "importpubkey": (2,), "importmulti":
    (0, 1), "verifychain": (0, 1), "pruneblockchain": (0,), "keypoolrefill": (0,), "getrawmempool": (0,),
    "estimatefee": (0,), "estimatesmartfee": (0,), "estimaterawfee": (0, 1), "prioritisetransaction": (1, 2),
    "setban": (2, 3), "setnetworkactive": (0,), "getmempoolancestors": (1,), "getmempooldescendants": (1,),
    "getblockhashes": (1, 2), "getspentinfo": (0,), "getaddresstxids": (0, 1), "getaddressbalance": (0, 1),
    "getaddressdeltas": (0,), "getaddressutxos": (0,), "getaddressmempool": (0, 1), "bumpfee": (1,), "logging":
    (0, 1), "disconnectnode": (1,), "echojson": (0, 1, 2, 3, 4, 5, 6, 7, 8, 9), "rescanblockchain": (0, 1),
    "listaddressesbyasset": (1, 2, 3), "listassetbalancesbyaddress": (1, 2, 3), "sendmessage": (2,),
    "requestsnapshot": (1,), "getsnapshotrequest": (1,), "listsnapshotrequests": (1,), "cancelsnapshotrequest":
    (1,), "distributereward": (1, 3), "getdistributestatus": (1, 3), "getsnapshot": (1,), "purgesnapshot": (1,),
    "stop": (0,), "getkawpowhash": (3,), "verifyheaders": (0,),
}
CONVERT = {(m, i) for m, ix in _CONVERT_POSITIONS.items() for i in ix}


class RPCClient:
    def __init__(self, host: str = "127.0.0.1", port: int = 19443, user: str | None = None,
                 password: str | None = None, cookie: str | None = None, timeout: float = 900,
                 wallet: str | None = None):
        self.host, self.port, self.timeout = host, port, timeout
        # -rpcwallet: wallet calls go to /wallet/<name> (multiwallet endpoint, src/wallet/rpcwallet.cpp)
        self.path = "/" if wallet is None else "/wallet/" + urllib.parse.quote(wallet)
        if cookie and os.path.exists(cookie) and not user:
            with open(cookie) as f:
                user, _, password = f.read().strip().partition(":")
        self.auth = None
        if user is not None:
            self.auth = "Basic " + base64.b64encode(f"{user}:{password or ''}".encode()).decode()
        self._id = 0

    def call_raw(self, payload) -> tuple[int, object]:
        conn = http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)
        headers = {"Content-Type": "application/json"}
        if self.auth:
            headers["Authorization"] = self.auth
        conn.request("POST", self.path, json.dumps(payload), headers)
        r = conn.getresponse()
        body = r.read()
        conn.close()
        if r.status == 401:
            raise PermissionError("incorrect rpcuser or rpcpassword (authorization failed)")
        return r.status, json.loads(body) if body else None

    def call(self, method: str, *params):
        self._id += 1
        _, rep = self.call_raw({"method": method, "params": list(params), "id": self._id})
        if rep.get("error"):
            e = rep["error"]
            raise RuntimeError(f"RPC error {e.get('code')}: {e.get('message')}")
        return rep["result"]

    def batch(self, calls: list[tuple[str, list]]):
        payload = [{"method": m, "params": p, "id": i} for i, (m, p) in enumerate(calls)]
        _, rep = self.call_raw(payload)
        return rep

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return lambda *p: self.call(name, *p)


def convert_params(method: str, args: list[str]):
    out = []
    for i, a in enumerate(args):
        if (method, i) in CONVERT:
            try:
                out.append(json.loads(a))
            except ValueError:
                raise SystemExit(f"Error parsing JSON:{a}")
        else:
            out.append(a)
    return out


def main(argv: list[str] | None = None) -> int:
    args = ArgsManager()
    rest = args.parse_parameters(sys.argv[1:] if argv is None else argv)
    if not rest:
        print("usage: nodexa-cli [options] <command> [params]", file=sys.stderr)
        return 1
    from ..chain.state import make_params

    params = make_params(args.network)
    datadir = os.path.expanduser(args.get("datadir", "~/.nodexa"))
    if args.network != "main":
        datadir = os.path.join(datadir, "testnet7" if args.network == "test" else "regtest")
    password = args.get("rpcpassword")
    stdin_lines = None
    if args.get_bool("stdinrpcpass", False):  # -stdinrpcpass: the password is the first stdin line
        stdin_lines = sys.stdin.read().split("\n")
        password = stdin_lines.pop(0)
    cli = RPCClient(args.get("rpcconnect", "127.0.0.1"), args.get_int("rpcport", params.default_rpc_port),
                    args.get("rpcuser"), password,
                    os.path.join(datadir, os.path.expanduser(args.get("rpccookiefile", ".cookie"))),
                    timeout=float(args.get_int("rpcclienttimeout", 900)), wallet=args.get("rpcwallet"))
    if args.get_bool("stdin", False):  # -stdin: one extra argument per input line
        lines = stdin_lines if stdin_lines is not None else sys.stdin.read().split("\n")
        rest = rest + (lines[:-1] if lines and lines[-1] == "" else lines)
    method, p = rest[0], rest[1:]
    if args.get_bool("named", False):
        named = {}
        for kv in p:
            k, _, v = kv.partition("=")
            try:
                named[k] = json.loads(v)
            except ValueError:
                named[k] = v
        req = {"method": method, "params": named, "id": 1}
    else:
        req = {"method": method, "params": convert_params(method, p), "id": 1}
    wait = args.get_bool("rpcwait", False)
    while True:  # -rpcwait: retry while the server is down or still warming up (CommandLineRPC)
        try:
            status, rep = cli.call_raw(req)
        except PermissionError as e:
            print(f"error: {e}", file=sys.stderr)
            return 1
        except (ConnectionError, OSError) as e:
            if not wait:
                print(f"error: couldn't connect to server: {e}", file=sys.stderr)
                return 87  # EXIT_FAILURE path of CConnectionFailed in the reference CLI
            time.sleep(1.0)
            continue
        if wait and (rep.get("error") or {}).get("code") == -28:  # RPC_IN_WARMUP
            time.sleep(1.0)
            continue
        break
    if rep.get("error"):
        e = rep["error"]
        print(f"error code: {e.get('code')}\nerror message:\n{e.get('message')}", file=sys.stderr)
        return abs(int(e.get("code", 1))) or 1
    res = rep.get("result")
    print(res if isinstance(res, str) else json.dumps(res, indent=2))
    return 0


if __name__ == "__main__":
    sys.exit(main())
