"""HTTP/1.1 JSON-RPC server with the reference's request semantics.

Parity:
  * HTTP front-end with a bounded work queue and N worker threads
    (src/httpserver.cpp:68-460, -rpcworkqueue / -rpcthreads, 503 "Work queue
    depth exceeded" when full), persistent connections.
  * Basic auth against -rpcuser/-rpcpassword, the `.cookie` file (src/httprpc.cpp:128,
    RPCAuthorized; GenerateAuthCookie, -rpccookiefile) or -rpcauth user:salt$hmac entries
    (multiUserAuthorized: HMAC-SHA256 keyed by the salt over the password).
  * -rpcallowip (ClientAllowed / InitHTTPAllowList: loopback always, then addresses and
    subnets as CIDR or netmask; 403 for the rest), -rpcthreads workers executing requests,
    -rpcservertimeout for idle keep-alive connections.
  * Single and batch requests (JSONRPCExecBatch, src/rpc/server.cpp:501),
    error -> HTTP status mapping (JSONErrorReply), warm-up gate (RPC_IN_WARMUP).
  * CRPCTable: category/name/handler/arg names, `help`, positional and named
    parameters (src/rpc/server.cpp:379-560).
The daemon runs this in-process next to the chain state and the GPU miner.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import ipaddress
import http.server
import json
import os
import queue
import secrets
import socketserver
import threading
import time
import urllib.parse
from dataclasses import dataclass
from typing import Callable

from ..utils import log
from .protocol import (REQUEST_WALLET, RPC_IN_WARMUP, RPC_INTERNAL_ERROR, RPC_INVALID_PARAMETER, RPC_INVALID_REQUEST,
                       RPC_METHOD_NOT_FOUND, RPC_PARSE_ERROR, RPCError, http_status_for, reply)


@dataclass
class RPCCommand:
    category: str
    name: str
    handler: Callable
    arg_names: tuple[str, ...]
    help: str = ""


# RPCs that call ObserveSafeMode() in the reference (src/wallet/rpcwallet.cpp, rpcdump.cpp,
# src/rpc/assets.cpp, messages.cpp, rawtransaction.cpp, rewards.cpp): refused while a safe-mode
# warning stands, unless -disablesafemode
SAFE_MODE_METHODS = frozenset((
    "sendtoaddress sendfromaddress listaddressgroupings getreceivedbyaddress getreceivedbyaccount getbalance "
    "getunconfirmedbalance move sendfrom sendmany listreceivedbyaddress listreceivedbyaccount listtransactions "
    "listaccounts listsinceblock gettransaction abandontransaction listlockunspent getwalletinfo listunspent "
    "fundrawtransaction abortrescan issue issueunique listassetbalancesbyaddress listmyassets transfer "
    "transferfromaddresses transferfromaddress reissue listassets issuequalifierasset issuerestrictedasset "
    "reissuerestrictedasset transferqualifier isvalidverifierstring sendmessage signrawtransaction "
    "sendrawtransaction testmempoolaccept distributereward getdistributestatus").split())


class RPCTable:
    def __init__(self) -> None:
        self.commands: dict[str, RPCCommand] = {}
        self.safe_mode: Callable[[], None] | None = None  # ObserveSafeMode (raises while in safe mode)
        self.warmup: str | None = None
        self.started = time.time()
        self.active: dict[int, tuple[str, float]] = {}
        self._lock = threading.Lock()

    def append(self, category: str, name: str, handler: Callable, arg_names=(), help: str = "") -> None:
        if name in self.commands:
            raise ValueError(f"duplicate RPC {name}")
        self.commands[name] = RPCCommand(category, name, handler, tuple(arg_names), help or (handler.__doc__ or ""))

    def help(self, name: str | None = None) -> str:
        if name:
            c = self.commands.get(name)
            if c is None:
                return f"help: unknown command: {name}"
            args = " ".join(f'"{a}"' for a in c.arg_names)
            return f"{c.name} {args}\n\n{c.help.strip()}"
        out, cat = [], None
        for c in sorted(self.commands.values(), key=lambda c: (c.category, c.name)):
            if c.category != cat:
                cat = c.category
                out.append(f"\n== {cat[0].upper() + cat[1:]} ==")
            out.append(f"{c.name} " + " ".join(f'"{a}"' for a in c.arg_names))
        return "\n".join(out).strip()

    def execute(self, method: str, params) -> object:
        if self.warmup is not None:
            raise RPCError(RPC_IN_WARMUP, self.warmup)
        cmd = self.commands.get(method)
        if cmd is None:
            raise RPCError(RPC_METHOD_NOT_FOUND, "Method not found")
        if self.safe_mode is not None and method in SAFE_MODE_METHODS:
            self.safe_mode()
        if isinstance(params, dict):  # named arguments
            unknown = set(params) - set(cmd.arg_names)
            if unknown:
                raise RPCError(RPC_INVALID_PARAMETER, f"Unknown named parameter {sorted(unknown)[0]}")
            last = max((cmd.arg_names.index(k) for k in params), default=-1)
            params = [params.get(a) for a in cmd.arg_names[:last + 1]]
        elif params is None:
            params = []
        elif not isinstance(params, list):
            raise RPCError(RPC_INVALID_REQUEST, "Params must be an array or object")
        tid = threading.get_ident()
        with self._lock:
            self.active[tid] = (method, time.time())
        try:
            return cmd.handler(params)
        finally:
            with self._lock:
                self.active.pop(tid, None)

    def exec_request(self, req: dict) -> dict:
        id_ = req.get("id") if isinstance(req, dict) else None
        try:
            if not isinstance(req, dict):
                raise RPCError(RPC_INVALID_REQUEST, "Invalid Request object")
            method = req.get("method")
            if not isinstance(method, str):
                raise RPCError(RPC_INVALID_REQUEST, "Method must be a string")
            log.log_print("rpc", f"ThreadRPCServer method={method}")
            return reply(self.execute(method, req.get("params")), None, id_)
        except RPCError as e:
            return reply(None, e.to_json(), id_)
        except Exception as e:  # handler bug or runtime error -> RPC_MISC style
            return reply(None, {"code": -1, "message": str(e)}, id_)


def parse_allow_subnets(specs: list[str]) -> list:
    """-rpcallowip values: an address, addr/prefix or addr/netmask (LookupSubNet)."""
    out = []
    for s in specs:
        try:
            out.append(ipaddress.ip_network(s.strip(), strict=False))
        except ValueError:
            raise ValueError(f"Invalid -rpcallowip subnet specification: {s}") from None
    return out


def ip_allowed(ip: str, nets: list) -> bool:
    try:
        a = ipaddress.ip_address(ip.split("%")[0])
    except ValueError:
        return False
    if a.is_loopback or (a.version == 6 and a.ipv4_mapped is not None and a.ipv4_mapped.is_loopback):
        return True
    if a.version == 6 and a.ipv4_mapped is not None:
        a = a.ipv4_mapped
    return any(a.version == n.version and a in n for n in nets)


def rpcauth_matches(entries: list[str], user: str, password: str) -> bool:
    """-rpcauth=<user>:<salt>$<hex hmac_sha256(key=salt, msg=password)>."""
    for e in entries:
        name, sep, rest = e.partition(":")
        salt, sep2, digest = rest.partition("$")
        if not sep or not sep2 or not hmac.compare_digest(name, user):
            continue
        want = hmac.new(salt.encode(), password.encode(), hashlib.sha256).hexdigest()
        if hmac.compare_digest(want, digest.lower()):
            return True
    return False


class _Handler(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "nodexa-json-rpc/0.1"

    def setup(self):
        self.timeout = self.server.idle_timeout  # -rpcservertimeout
        super().setup()

    def handle_one_request(self):
        if not self.server.client_allowed(self.client_address[0]):  # http_request_cb: ClientAllowed
            log.log_print("http", f"HTTP request from {self.client_address[0]} rejected: not in -rpcallowip")
            self.close_connection = True
            try:
                self.raw_requestline = self.rfile.readline(65537)
                self.send_response(403)
                self.send_header("Content-Length", "0")
                self.end_headers()
            except OSError:
                pass
            return
        try:
            super().handle_one_request()
        except TimeoutError:
            self.close_connection = True

    def log_message(self, fmt, *args):  # route to category logging
        log.log_print("http", fmt % args)

    def _send(self, status: int, body: bytes, ctype: str = "application/json") -> None:
        self.send_response(status)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _authorized(self) -> bool:
        auth = self.headers.get("Authorization", "")
        if not auth.startswith("Basic "):
            return False
        try:
            userpass = base64.b64decode(auth[6:].strip()).decode()
        except Exception:
            return False
        if any(hmac.compare_digest(userpass, c) for c in self.server.credentials):
            return True
        user, _, pw = userpass.partition(":")
        return rpcauth_matches(self.server.rpcauth, user, pw)

    def _same_origin_or_cli(self) -> bool:
        """CSRF guard. A browser that holds the RPC credentials (Basic auth remembered
        after opening /gui) would attach them to a cross-site form POST (enctype=text/plain) or to a
        page's fetch(). Browsers mark such requests with Origin / Referer / Sec-Fetch-* headers;
        command-line clients (nodexa-cli, curl, the reference's clore-cli) send none of them and
        pass as before. A browser request must come from this server's own origin AND carry the
        per-process token that only the served /gui page holds (a custom header: a cross-site form
        cannot set one, and a cross-site fetch() with one needs a CORS preflight this server never
        grants)."""
        h = self.headers
        if not any(h.get(k) for k in ("Origin", "Referer", "Sec-Fetch-Site", "Sec-Fetch-Mode")):
            return True
        src = h.get("Origin") or h.get("Referer") or ""
        if src and src != "null":
            same = urllib.parse.urlsplit(src).netloc == h.get("Host", "")
        else:
            same = h.get("Sec-Fetch-Site") in ("same-origin", "none")
        return same and hmac.compare_digest(h.get("X-Nodexa-CSRF", ""), self.server.csrf_token)

    def do_POST(self):  # noqa: N802
        srv: RPCHTTPServer = self.server
        if (srv.credentials or srv.rpcauth) and not self._authorized():
            log.log_printf(f"ThreadRPCServer incorrect password attempt from {self.client_address[0]}")
            time.sleep(0.25)
            self.send_response(401)
            self.send_header("WWW-Authenticate", 'Basic realm="jsonrpc"')
            self.send_header("Content-Length", "0")
            self.end_headers()
            return
        if not self._same_origin_or_cli():
            log.log_printf(f"JSON-RPC POST from {self.client_address[0]} rejected: browser request without the "
                           f"web wallet's token (Origin {self.headers.get('Origin')!r})")
            self._send(403, b"Forbidden: cross-site request", "text/plain")
            return
        if not srv.slots.acquire(blocking=False):
            self._send(503, b"Work queue depth exceeded", "text/plain")
            return
        path = self.path.split("?")[0]
        if path != "/" and not path.startswith("/wallet/"):  # the two JSON-RPC handlers the reference registers
            srv.slots.release()
            self._send(404, b"", "text/plain")
            return
        srv.workers.acquire()  # -rpcthreads: requests past the work queue wait for a worker
        token = REQUEST_WALLET.set(urllib.parse.unquote(path[len("/wallet/"):]) if path != "/" else "")
        try:
            length = int(self.headers.get("Content-Length", "0"))
            raw = self.rfile.read(length)
            try:
                req = json.loads(raw)
            except ValueError:
                body = json.dumps(reply(None, {"code": RPC_PARSE_ERROR, "message": "Parse error"}, None))
                self._send(500, body.encode())
                return
            if isinstance(req, list):
                body = json.dumps([srv.table.exec_request(r) for r in req])
                self._send(200, body.encode())
                return
            rep = srv.table.exec_request(req)
            status = 200 if rep["error"] is None else http_status_for(rep["error"]["code"])
            self._send(status, json.dumps(rep).encode())
        finally:
            REQUEST_WALLET.reset(token)
            srv.workers.release()
            srv.slots.release()

    def do_GET(self):  # noqa: N802
        # the web wallet (gui/index.html, the Qt GUI's role): behind the RPC credentials like the
        # JSON-RPC endpoint it talks to
        if self.path.split("?")[0] in ("/gui", "/gui/", "/gui/index.html") and self.server.gui is not None:
            srv = self.server
            if (srv.credentials or srv.rpcauth) and not self._authorized():
                self.send_response(401)
                self.send_header("WWW-Authenticate", 'Basic realm="jsonrpc"')
                self.send_header("Content-Length", "0")
                self.end_headers()
                return
            with open(srv.gui, "rb") as f:
                page = f.read().replace(b"__NODEXA_CSRF__", srv.csrf_token.encode())
            self.send_response(200)
            self.send_header("Content-Type", "text/html; charset=utf-8")
            self.send_header("Content-Length", str(len(page)))
            self.send_header("Cache-Control", "no-store")  # the token is per process
            self.send_header("X-Frame-Options", "DENY")
            self.end_headers()
            self.wfile.write(page)
            return
        # REST subset (src/rest.cpp:569-580): /rest/chaininfo.json
        if self.path.startswith("/rest/") and self.server.rest is not None:
            try:
                status, ctype, body = self.server.rest(self.path)
            except Exception as e:
                status, ctype, body = 400, "text/plain", str(e).encode()
            self._send(status, body, ctype)
            return
        if self.path.startswith("/rest/"):  # -rest off: no handler registered for the prefix
            self._send(404, b"", "text/plain")
            return
        self._send(405, b"JSONRPC server handles only POST requests", "text/plain")


class RPCHTTPServer(socketserver.ThreadingMixIn, http.server.HTTPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, addr, table: RPCTable, credentials: list[str], work_queue: int, rest=None,
                 rpcauth: list[str] | None = None, allow: list | None = None, threads: int = 4,
                 idle_timeout: float = 30.0, gui: str | None = None):
        super().__init__(addr, _Handler)
        self.gui = gui  # path of the web wallet page, or None (-webgui=0, the default)
        self.csrf_token = secrets.token_hex(16)  # handed to the /gui page; required on browser POSTs
        self.table = table
        self.credentials = credentials
        self.rpcauth = list(rpcauth or [])
        self.allow = list(allow or [])
        # -rpcworkqueue bounds the requests admitted (queued + running); -rpcthreads the running
        self.slots = threading.BoundedSemaphore(max(1, work_queue) + max(1, threads))
        self.workers = threading.BoundedSemaphore(max(1, threads))
        self.idle_timeout = idle_timeout
        self.rest = rest

    def client_allowed(self, ip: str) -> bool:
        return ip_allowed(ip, self.allow)


def cookie_path(datadir: str, cookiefile: str | None = None) -> str:
    """GetAuthCookieFile: -rpccookiefile (relative to the data directory) or <datadir>/.cookie."""
    return os.path.join(datadir, os.path.expanduser(cookiefile or ".cookie"))


def make_cookie(datadir: str, cookiefile: str | None = None) -> str:
    """GenerateAuthCookie: `__cookie__:<64 hex>` in the cookie file (0600)."""
    token = "__cookie__:" + secrets.token_hex(32)
    path = cookie_path(datadir, cookiefile)
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w") as f:
        f.write(token)
    return token


def delete_cookie(datadir: str, cookiefile: str | None = None) -> None:
    try:
        os.unlink(cookie_path(datadir, cookiefile))
    except OSError:
        pass


class RPCServer:
    def __init__(self, table: RPCTable, host: str, port: int, credentials: list[str], work_queue: int = 16,
                 rest=None, **kw):
        self.httpd = RPCHTTPServer((host, port), table, credentials, work_queue, rest, **kw)
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, name="http", daemon=True)

    def start(self) -> None:
        self.thread.start()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
