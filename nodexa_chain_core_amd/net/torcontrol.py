"""Tor control-port client: an ephemeral onion service for the P2P port.

Parity (behaviour): src/torcontrol.cpp —
* reply framing `<code>(-|+| )<data>` with `+` data blocks ended by "." and 6xx async replies
  (TorControlConnection::readcb, :136-190);
* `SplitTorReplyLine` / `ParseTorReplyMapping` (:259-363), including QuotedString C escapes and
  octals, checked against src/test/torcontrol_tests.cpp;
* TorController (:416-727): PROTOCOLINFO 1, then AUTHENTICATE with -torpassword
  (HASHEDPASSWORD), NULL, or SAFECOOKIE (AUTHCHALLENGE with a 32-byte client nonce; the server
  hash is checked with HMAC-SHA256 keyed by "Tor safe cookie authentication
  server-to-controller hash", the client answers with the controller-to-server key); then, unless
  -onion is given, the onion proxy defaults to 127.0.0.1:9050; ADD_ONION <key|NEW:RSA1024>
  Port=<p>,127.0.0.1:<p>; the key persists in <datadir>/onion_private_key and the service is
  advertised as a local address (AddLocal) until the control connection drops (RemoveLocal);
  reconnects back off from 1 s by x1.5.
The reference drives this from libevent callbacks; here one daemon thread runs the exchange
with blocking sockets, which is all a single control connection needs.
"""
from __future__ import annotations

import hashlib
import hmac
import os
import socket
import threading

from ..utils import log
from .netbase import Proxy, parse_host_port

DEFAULT_TOR_CONTROL = "127.0.0.1:9051"
TOR_COOKIE_SIZE = 32
TOR_NONCE_SIZE = 32
TOR_SAFE_SERVERKEY = b"Tor safe cookie authentication server-to-controller hash"
TOR_SAFE_CLIENTKEY = b"Tor safe cookie authentication controller-to-server hash"
RECONNECT_TIMEOUT_START = 1.0
RECONNECT_TIMEOUT_EXP = 1.5


def split_reply_line(s: str) -> tuple[str, str]:
    """'AUTH METHODS=...' -> ('AUTH', 'METHODS=...'); only the first space separates."""
    head, sep, rest = s.partition(" ")
    return head, rest if sep else ""


def _unescape(value: str) -> str:
    out, i = [], 0
    while i < len(value):
        c = value[i]
        if c != "\\":
            out.append(c)
            i += 1
            continue
        i += 1
        c = value[i]
        if c in "ntr":
            out.append({"n": "\n", "t": "\t", "r": "\r"}[c])
            i += 1
        elif "0" <= c <= "7":
            j = 1
            while j < 3 and i + j < len(value) and "0" <= value[i + j] <= "7":
                j += 1
            if j == 3 and c > "3":  # Tor limits a three-digit octal to \377
                j -= 1
            out.append(chr(int(value[i:i + j], 8)))
            i += j
        else:
            out.append(c)
            i += 1
    return "".join(out)


def parse_reply_mapping(s: str) -> dict[str, str]:
    """'KEY=VALUE KEY="quoted value" ...' -> dict; {} on a malformed line. A bare word where a
    key is expected starts the OptArguments tail, which carries no data and is dropped."""
    out: dict[str, str] = {}
    p, n = 0, len(s)
    while p < n:
        k0 = p
        while p < n and s[p] not in "= ":
            p += 1
        if p == n:
            return {}
        if s[p] == " ":
            break
        key = s[k0:p]
        p += 1
        if p < n and s[p] == '"':
            p += 1
            v0, escape = p, False
            while p < n and (escape or s[p] != '"'):
                escape = s[p] == "\\" and not escape
                p += 1
            if p == n:
                return {}
            value = _unescape(s[v0:p])
            p += 1
        else:
            v0 = p
            while p < n and s[p] != " ":
                p += 1
            value = s[v0:p]
        if p < n and s[p] == " ":
            p += 1
        out[key] = value
    return out


class TorControlConnection:
    """One control-port connection: send a command, read its complete reply."""

    def __init__(self, host: str, port: int, timeout: float = 10.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.settimeout(None)
        self._buf = b""

    def _line(self) -> str:
        while b"\r\n" not in self._buf:
            chunk = self.sock.recv(4096)
            if not chunk:
                raise ConnectionError("tor control connection closed")
            self._buf += chunk
        line, _, self._buf = self._buf.partition(b"\r\n")
        return line.decode("latin-1")

    def read_reply(self) -> tuple[int, list[str]]:
        """The next synchronous reply (code, lines); asynchronous 6xx events are skipped."""
        while True:
            code, lines = 0, []
            while True:
                s = self._line()
                if len(s) < 4:
                    continue
                code = int(s[:3])
                if s[3] == "+":  # data block: the lines up to "." belong to this reply line
                    data = [s[4:]]
                    while True:
                        d = self._line()
                        if d == ".":
                            break
                        data.append(d[1:] if d.startswith("..") else d)
                    lines.append("\n".join(data))
                    continue
                lines.append(s[4:])
                if s[3] == " ":
                    break
            if code < 600:
                return code, lines

    def command(self, cmd: str) -> tuple[int, list[str]]:
        self.sock.sendall(cmd.encode("latin-1") + b"\r\n")
        return self.read_reply()

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


def compute_response(key: bytes, cookie: bytes, client_nonce: bytes, server_nonce: bytes) -> bytes:
    return hmac.new(key, cookie + client_nonce + server_nonce, hashlib.sha256).digest()


class TorController:
    """Keeps an ephemeral onion service for `listen_port` while a Tor control port is reachable."""

    def __init__(self, target: str, datadir: str | None, listen_port: int, proxies=None,
                 add_local=None, remove_local=None, password: str = "", onion_arg_set: bool = False):
        self.host, self.port = parse_host_port(target, 9051)
        self.datadir = datadir
        self.listen_port = listen_port
        self.proxies = proxies
        self.add_local = add_local or (lambda host, port: None)
        self.remove_local = remove_local or (lambda host, port: None)
        self.password = password
        self.onion_arg_set = onion_arg_set
        self.service: str | None = None
        self.private_key = ""
        self.reconnect_timeout = RECONNECT_TIMEOUT_START
        self.last_error = ""
        self._stop = threading.Event()
        self._conn: TorControlConnection | None = None
        self._thread: threading.Thread | None = None
        pk = self.private_key_file()
        if pk and os.path.exists(pk):
            with open(pk, "r", encoding="latin-1") as f:
                self.private_key = f.read()

    def private_key_file(self) -> str | None:
        return os.path.join(self.datadir, "onion_private_key") if self.datadir else None

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        self._thread = threading.Thread(target=self._run, name="torcontrol", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._conn is not None:
            self._conn.close()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                self._conn = TorControlConnection(self.host, self.port)
            except OSError as e:
                self.last_error = f"Not connected to Tor control port {self.host}:{self.port}: {e}"
                log.log_print("tor", f"tor: {self.last_error}, trying to reconnect")
                self._backoff()
                continue
            try:
                self.reconnect_timeout = RECONNECT_TIMEOUT_START
                self.session(self._conn)
                self._conn.read_reply()  # hold the connection: the service lives as long as it
            except (OSError, ConnectionError, ValueError) as e:
                self.last_error = str(e)
            finally:
                self._conn.close()
                if self.service:  # disconnected: the onion address is no longer ours
                    self.remove_local(self.service, self.listen_port)
                    self.service = None
            if not self._stop.is_set():
                log.log_print("tor", "tor: Not connected to Tor control port, trying to reconnect")
                self._backoff()

    def _backoff(self) -> None:
        self._stop.wait(self.reconnect_timeout)
        self.reconnect_timeout *= RECONNECT_TIMEOUT_EXP

    # ------------------------------------------------------------------ protocol
    def session(self, conn: TorControlConnection) -> str | None:
        """PROTOCOLINFO -> authenticate -> ADD_ONION. Returns the service name or None."""
        code, lines = conn.command("PROTOCOLINFO 1")
        if code != 250:
            raise ValueError("tor: Requesting protocol info failed")
        methods, cookiefile = set(), ""
        for line in lines:
            kind, rest = split_reply_line(line)
            if kind == "AUTH":
                m = parse_reply_mapping(rest)
                methods = set(m.get("METHODS", "").split(","))
                cookiefile = m.get("COOKIEFILE", "")
            elif kind == "VERSION":
                log.log_print("tor", f"tor: Connected to Tor version {parse_reply_mapping(rest).get('Tor', '')}")
        if self.password:
            if "HASHEDPASSWORD" not in methods:
                raise ValueError("tor: Password provided with -torpassword, but HASHEDPASSWORD "
                                 "authentication is not available")
            code, _ = conn.command(f'AUTHENTICATE "{self.password}"')
        elif "NULL" in methods:
            code, _ = conn.command("AUTHENTICATE")
        elif "SAFECOOKIE" in methods:
            with open(cookiefile, "rb") as f:
                cookie = f.read(TOR_COOKIE_SIZE + 1)
            if len(cookie) != TOR_COOKIE_SIZE:
                raise ValueError(f"tor: Authentication cookie {cookiefile} is not exactly {TOR_COOKIE_SIZE} bytes")
            client_nonce = os.urandom(TOR_NONCE_SIZE)
            code, lines = conn.command("AUTHCHALLENGE SAFECOOKIE " + client_nonce.hex())
            kind, rest = split_reply_line(lines[0] if lines else "")
            if code != 250 or kind != "AUTHCHALLENGE":
                raise ValueError("tor: SAFECOOKIE authentication challenge failed")
            m = parse_reply_mapping(rest)
            server_hash = bytes.fromhex(m.get("SERVERHASH", ""))
            server_nonce = bytes.fromhex(m.get("SERVERNONCE", ""))
            if len(server_nonce) != TOR_NONCE_SIZE:
                raise ValueError("tor: ServerNonce is not 32 bytes, as required by spec")
            want = compute_response(TOR_SAFE_SERVERKEY, cookie, client_nonce, server_nonce)
            if not hmac.compare_digest(want, server_hash):
                raise ValueError("tor: ServerHash is not as expected")
            code, _ = conn.command("AUTHENTICATE " +
                                   compute_response(TOR_SAFE_CLIENTKEY, cookie, client_nonce, server_nonce).hex())
        else:
            raise ValueError("tor: No supported authentication method")
        if code != 250:
            raise ValueError("tor: Authentication failed")
        log.log_print("tor", "tor: Authentication successful")
        if not self.onion_arg_set and self.proxies is not None:  # Tor's SOCKS port serves .onion
            self.proxies.set_proxy("onion", Proxy("127.0.0.1", 9050, True))
            self.proxies.set_limited("onion", False)
        key = self.private_key or "NEW:RSA1024"
        code, lines = conn.command(f"ADD_ONION {key} Port={self.listen_port},127.0.0.1:{self.listen_port}")
        if code != 250:
            raise ValueError("tor: Add onion failed")
        m: dict[str, str] = {}
        for line in lines:
            m.update(parse_reply_mapping(line))
        if "ServiceID" not in m:
            raise ValueError("tor: Error parsing ADD_ONION parameters")
        self.service = m["ServiceID"] + ".onion"
        if "PrivateKey" in m:
            self.private_key = m["PrivateKey"]
            pk = self.private_key_file()
            if pk:
                with open(pk, "w", encoding="latin-1") as f:
                    f.write(self.private_key)
                log.log_print("tor", f"tor: Cached service private key to {pk}")
        log.log_printf(f"tor: Got service ID {m['ServiceID']}, advertising service {self.service}:{self.listen_port}")
        self.add_local(self.service, self.listen_port)
        return self.service
