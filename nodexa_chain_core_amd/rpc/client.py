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

from ..utils.config import ArgsManager

# (method, param index) pairs whose CLI strings are parsed as JSON
CONVERT = {
    ("generate", 0), ("generate", 1), ("generatetoaddress", 0), ("generatetoaddress", 2),
    ("getblockhash", 0), ("getblock", 1), ("getblockheader", 1), ("getnetworkhashps", 0), ("getnetworkhashps", 1),
    ("getblocktemplate", 0), ("setgenerate", 0), ("setgenerate", 1), ("getkawpowhash", 3),
    ("prioritisetransaction", 1), ("prioritisetransaction", 2), ("waitfornewblock", 0), ("verifychain", 0),
    ("verifychain", 1), ("logging", 0), ("logging", 1), ("getrawmempool", 0), ("verifyheaders", 0),
    ("sendrawtransaction", 1),
}


class RPCClient:
    def __init__(self, host: str = "127.0.0.1", port: int = 19443, user: str | None = None,
                 password: str | None = None, cookie: str | None = None, timeout: float = 900):
        self.host, self.port, self.timeout = host, port, timeout
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
        conn.request("POST", "/", json.dumps(payload), headers)
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
    cli = RPCClient(args.get("rpcconnect", "127.0.0.1"), args.get_int("rpcport", params.default_rpc_port),
                    args.get("rpcuser"), args.get("rpcpassword"),
                    os.path.join(datadir, os.path.expanduser(args.get("rpccookiefile", ".cookie"))),
                    timeout=float(args.get_int("rpcclienttimeout", 900)))
    if args.get_bool("stdin", False):  # -stdin: one extra argument per input line
        rest = rest + [line.rstrip("\n") for line in sys.stdin]
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
