"""Tor control client and SOCKS5 proxying (netbase part of N1).

The reply parsers are checked against every vector of the reference's
src/test/torcontrol_tests.cpp. The controller runs against an in-process fake Tor control port
(PROTOCOLINFO, AUTHCHALLENGE SAFECOOKIE with the real HMAC exchange, AUTHENTICATE, ADD_ONION),
and outbound P2P connections go through an in-process SOCKS5 server (RFC 1928 / 1929) that
relays to a second node. No Tor binary exists in this environment, so the fakes speak the
protocol as control-spec and the reference describe it; parity with a live Tor is unpinned."""
import hashlib
import hmac
import os
import socket
import struct
import threading
import time

import pytest

from nodexa_chain_core_amd.net import netbase, torcontrol as tc
from test_node_rpc import client, node_factory  # noqa: F401 — shared fixtures

SPLIT = [
    ("PROTOCOLINFO PIVERSION", "PROTOCOLINFO", "PIVERSION"),
    ('AUTH METHODS=COOKIE,SAFECOOKIE COOKIEFILE="/home/x/.tor/control_auth_cookie"', "AUTH",
     'METHODS=COOKIE,SAFECOOKIE COOKIEFILE="/home/x/.tor/control_auth_cookie"'),
    ("AUTH METHODS=NULL", "AUTH", "METHODS=NULL"),
    ("AUTH METHODS=HASHEDPASSWORD", "AUTH", "METHODS=HASHEDPASSWORD"),
    ('VERSION Tor="0.2.9.8 (git-a0df013ea241b026)"', "VERSION", 'Tor="0.2.9.8 (git-a0df013ea241b026)"'),
    ("AUTHCHALLENGE SERVERHASH=aaaa SERVERNONCE=bbbb", "AUTHCHALLENGE", "SERVERHASH=aaaa SERVERNONCE=bbbb"),
    ("COMMAND", "COMMAND", ""),
    ("COMMAND SOME  ARGS", "COMMAND", "SOME  ARGS"),
    ("COMMAND  ARGS", "COMMAND", " ARGS"),
    ("COMMAND   EVEN+more  ARGS", "COMMAND", "  EVEN+more  ARGS"),
]

MAPPING = [
    ('METHODS=COOKIE,SAFECOOKIE COOKIEFILE="/home/x/.tor/control_auth_cookie"',
     {"METHODS": "COOKIE,SAFECOOKIE", "COOKIEFILE": "/home/x/.tor/control_auth_cookie"}),
    ("METHODS=NULL", {"METHODS": "NULL"}),
    ("METHODS=HASHEDPASSWORD", {"METHODS": "HASHEDPASSWORD"}),
    ('Tor="0.2.9.8 (git-a0df013ea241b026)"', {"Tor": "0.2.9.8 (git-a0df013ea241b026)"}),
    ("SERVERHASH=aaaa SERVERNONCE=bbbb", {"SERVERHASH": "aaaa", "SERVERNONCE": "bbbb"}),
    ("ServiceID=exampleonion1234", {"ServiceID": "exampleonion1234"}),
    ("PrivateKey=RSA1024:BLOB", {"PrivateKey": "RSA1024:BLOB"}),
    ("ClientAuth=bob:BLOB", {"ClientAuth": "bob:BLOB"}),
    ("Foo=Bar=Baz Spam=Eggs", {"Foo": "Bar=Baz", "Spam": "Eggs"}),
    ('Foo="Bar=Baz"', {"Foo": "Bar=Baz"}),
    ('Foo="Bar Baz"', {"Foo": "Bar Baz"}),
    ('Foo="Bar\\ Baz"', {"Foo": "Bar Baz"}),
    ('Foo="Bar\\Baz"', {"Foo": "BarBaz"}),
    ('Foo="Bar\\@Baz"', {"Foo": "Bar@Baz"}),
    ('Foo="Bar\\"Baz" Spam="\\"Eggs\\""', {"Foo": 'Bar"Baz', "Spam": '"Eggs"'}),
    ('Foo="Bar\\\\Baz"', {"Foo": "Bar\\Baz"}),
    ('Foo="Bar\\nBaz\\t" Spam="\\rEggs" Octals="\\1a\\11\\17\\18\\81\\377\\378\\400\\2222" Final=Check',
     {"Foo": "Bar\nBaz\t", "Spam": "\rEggs", "Octals": "\1a\11\17\1" "881\377\37" "8\40" "0\222" "2",
      "Final": "Check"}),
    ('Valid=Mapping Escaped="Escape\\\\"', {"Valid": "Mapping", "Escaped": "Escape\\"}),
    ('Valid=Mapping Bare="Escape\\"', {}),
    ('OneOctal="OneEnd\\1" TwoOctal="TwoEnd\\11"', {"OneOctal": "OneEnd\1", "TwoOctal": "TwoEnd\11"}),
    ('Null="\\0"', {"Null": "\0"}),
    ("SOME=args,here MORE optional=arguments  here", {"SOME": "args,here"}),
    ("ARGS", {}), ("MORE ARGS", {}), ("MORE  ARGS", {}), ("EVEN more=ARGS", {}), ("EVEN+more ARGS", {}),
]


@pytest.mark.parametrize("line,kind,args", SPLIT)
def test_split_reply_line_reference_vectors(line, kind, args):
    assert tc.split_reply_line(line) == (kind, args)


@pytest.mark.parametrize("line,expected", MAPPING)
def test_parse_reply_mapping_reference_vectors(line, expected):
    assert tc.parse_reply_mapping(line) == expected


# ---------------------------------------------------------------------------- fake Tor control port
class FakeTor:
    def __init__(self, tmp_path, methods="SAFECOOKIE", password="", bad_server_hash=False):
        self.methods, self.password, self.bad_server_hash = methods, password, bad_server_hash
        self.cookie = os.urandom(32)
        self.cookiefile = str(tmp_path / "control_auth_cookie")
        with open(self.cookiefile, "wb") as f:
            f.write(self.cookie)
        self.commands: list[str] = []
        self.authenticated = False
        self.srv = socket.socket()
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(4)
        self.port = self.srv.getsockname()[1]
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        while True:
            try:
                conn, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._session, args=(conn,), daemon=True).start()

    def _session(self, conn):
        f = conn.makefile("rb")
        client_nonce = server_nonce = None
        while True:
            line = f.readline()
            if not line:
                return
            cmd = line.decode().rstrip("\r\n")
            self.commands.append(cmd)
            send = lambda s: conn.sendall(s.encode())  # noqa: E731
            if cmd == "PROTOCOLINFO 1":
                send('650 STATUS_GENERAL NOTICE async event, never inside a reply\r\n'
                     f'250-PROTOCOLINFO 1\r\n250-AUTH METHODS={self.methods} COOKIEFILE="{self.cookiefile}"\r\n'
                     '250-VERSION Tor="0.4.8.9"\r\n250 OK\r\n')
            elif cmd.startswith("AUTHCHALLENGE SAFECOOKIE "):
                client_nonce = bytes.fromhex(cmd.split()[2])
                server_nonce = os.urandom(32)
                h = hmac.new(tc.TOR_SAFE_SERVERKEY, self.cookie + client_nonce + server_nonce, hashlib.sha256).digest()
                if self.bad_server_hash:
                    h = bytes(32)
                send(f"250 AUTHCHALLENGE SERVERHASH={h.hex().upper()} SERVERNONCE={server_nonce.hex().upper()}\r\n")
            elif cmd.startswith("AUTHENTICATE"):
                arg = cmd[len("AUTHENTICATE"):].strip()
                if "NULL" in self.methods:
                    ok = arg == ""
                elif "HASHEDPASSWORD" in self.methods:
                    ok = arg == f'"{self.password}"'
                else:
                    want = hmac.new(tc.TOR_SAFE_CLIENTKEY, self.cookie + client_nonce + server_nonce,
                                    hashlib.sha256).hexdigest()
                    ok = arg.lower() == want
                self.authenticated = ok
                send("250 OK\r\n" if ok else "515 Authentication failed\r\n")
            elif cmd.startswith("ADD_ONION ") and self.authenticated:
                key = cmd.split()[1]
                out = "250-ServiceID=abcdefghijklmnop\r\n"
                if key.startswith("NEW:"):
                    out += "250-PrivateKey=RSA1024:SECRETBLOB\r\n"
                send(out + "250 OK\r\n")
            else:
                send("510 Unrecognized command\r\n")

    def close(self):
        self.srv.close()


@pytest.mark.parametrize("methods,password", [("COOKIE,SAFECOOKIE", ""), ("NULL", ""), ("HASHEDPASSWORD", "s3cret")])
def test_controller_authenticates_and_adds_onion(tmp_path, methods, password):
    tor = FakeTor(tmp_path, methods, password)
    added = []
    proxies = netbase.ProxyTable()
    ctl = tc.TorController(f"127.0.0.1:{tor.port}", str(tmp_path), 19444, proxies=proxies,
                           add_local=lambda h, p: added.append((h, p)), password=password)
    conn = tc.TorControlConnection("127.0.0.1", tor.port)
    try:
        assert ctl.session(conn) == "abcdefghijklmnop.onion"
    finally:
        conn.close()
    assert added == [("abcdefghijklmnop.onion", 19444)]
    assert tor.commands[-1] == "ADD_ONION NEW:RSA1024 Port=19444,127.0.0.1:19444"
    with open(tmp_path / "onion_private_key") as f:
        assert f.read() == "RSA1024:SECRETBLOB"
    assert str(proxies.get_proxy("onion")) == "127.0.0.1:9050" and proxies.is_reachable("onion")
    # a restarted controller re-uses the cached key instead of asking for a new one
    ctl2 = tc.TorController(f"127.0.0.1:{tor.port}", str(tmp_path), 19444, password=password)
    conn = tc.TorControlConnection("127.0.0.1", tor.port)
    try:
        ctl2.session(conn)
    finally:
        conn.close()
    assert tor.commands[-1] == "ADD_ONION RSA1024:SECRETBLOB Port=19444,127.0.0.1:19444"
    tor.close()


def test_controller_rejects_a_wrong_server_hash(tmp_path):
    tor = FakeTor(tmp_path, "SAFECOOKIE", bad_server_hash=True)
    ctl = tc.TorController(f"127.0.0.1:{tor.port}", str(tmp_path), 19444)
    conn = tc.TorControlConnection("127.0.0.1", tor.port)
    with pytest.raises(ValueError, match="ServerHash is not as expected"):
        ctl.session(conn)
    conn.close()
    assert not any(c.startswith("AUTHENTICATE") for c in tor.commands)
    tor.close()
    with pytest.raises(ValueError, match="HASHEDPASSWORD"):
        tor2 = FakeTor(tmp_path, "NULL")
        conn = tc.TorControlConnection("127.0.0.1", tor2.port)
        try:
            tc.TorController("x", None, 1, password="pw").session(conn)
        finally:
            conn.close()
            tor2.close()


def test_node_advertises_its_onion_service(core, node_factory, tmp_path):  # noqa: F811
    tor = FakeTor(tmp_path, "SAFECOOKIE")
    node, _ = node_factory(("-listen=1", "-port=0", f"-torcontrol=127.0.0.1:{tor.port}"))
    c = client(node)
    deadline = time.time() + 10
    while time.time() < deadline:
        info = c.getnetworkinfo()
        if any(a["address"].endswith(".onion") for a in info["localaddresses"]):
            break
        time.sleep(0.1)
    onion = [a for a in info["localaddresses"] if a["address"].endswith(".onion")]
    assert onion and onion[0]["address"] == "abcdefghijklmnop.onion" and onion[0]["port"] == node.connman.port
    nets = {n["name"]: n for n in info["networks"]}
    assert nets["onion"]["reachable"] and nets["onion"]["proxy"] == "127.0.0.1:9050"
    assert os.path.exists(os.path.join(node.datadir, "onion_private_key"))
    tor.close()


# ---------------------------------------------------------------------------- SOCKS5
class FakeSocks5:
    """RFC 1928 server with optional RFC 1929 login that relays CONNECTs to 127.0.0.1:<port>
    (every destination name resolves there) or answers with `fail_code`."""

    def __init__(self, fail_code=0):
        self.fail_code = fail_code
        self.requests: list[tuple] = []
        self.srv = socket.socket()
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(8)
        self.port = self.srv.getsockname()[1]
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        while True:
            try:
                conn, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._one, args=(conn,), daemon=True).start()

    @staticmethod
    def _read(c, n):
        b = b""
        while len(b) < n:
            x = c.recv(n - len(b))
            if not x:
                raise OSError("eof")
            b += x
        return b

    def _one(self, c):
        try:
            ver, nm = self._read(c, 2)
            methods = self._read(c, nm)
            cred = None
            if 2 in methods:
                c.sendall(b"\x05\x02")
                _, ul = self._read(c, 2)
                user = self._read(c, ul)
                pl = self._read(c, 1)[0]
                pw = self._read(c, pl)
                cred = (user.decode(), pw.decode())
                c.sendall(b"\x01\x00")
            else:
                c.sendall(b"\x05\x00")
            _, cmd, _, atyp = self._read(c, 4)
            host = self._read(c, self._read(c, 1)[0]).decode()
            port = struct.unpack(">H", self._read(c, 2))[0]
            self.requests.append((host, port, cred))
            if self.fail_code:
                c.sendall(bytes([5, self.fail_code, 0, 1]) + bytes(6))
                c.close()
                return
            up = socket.create_connection(("127.0.0.1", port))
            c.sendall(b"\x05\x00\x00\x01" + bytes(4) + b"\x00\x00")
            for a, b in ((c, up), (up, c)):
                threading.Thread(target=self._pipe, args=(a, b), daemon=True).start()
        except OSError:
            c.close()

    @staticmethod
    def _pipe(a, b):
        try:
            while True:
                d = a.recv(65536)
                if not d:
                    break
                b.sendall(d)
        except OSError:
            pass
        finally:
            for s in (a, b):
                try:
                    s.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass

    def close(self):
        self.srv.close()


def test_socks5_connect_and_errors():
    echo = socket.socket()
    echo.bind(("127.0.0.1", 0))
    echo.listen(1)

    def _echo():
        s, _ = echo.accept()
        s.sendall(s.recv(5))
        s.close()
    threading.Thread(target=_echo, daemon=True).start()
    px = FakeSocks5()
    table = netbase.ProxyTable()
    table.set_proxy("ipv4", netbase.Proxy("127.0.0.1", px.port, True))
    s = table.connect("peer.example", echo.getsockname()[1])
    s.sendall(b"hello")
    assert s.recv(5) == b"hello"
    s.close()
    host, port, cred = px.requests[0]
    assert host == "peer.example" and port == echo.getsockname()[1] and cred and cred[0] == cred[1]
    bad = FakeSocks5(fail_code=5)
    table.set_proxy("ipv4", netbase.Proxy("127.0.0.1", bad.port, False))
    with pytest.raises(netbase.ProxyError, match="connection refused"):
        table.connect("10.1.2.3", 1)
    assert bad.requests[0][2] is None  # no randomized credentials: no-auth greeting only
    with pytest.raises(ConnectionError, match="not reachable"):
        table.connect("abcdefghijklmnop.onion", 1)  # no onion proxy configured
    assert netbase.network_of("::1") == "ipv6" and netbase.parse_host_port("[::1]:8", 1) == ("::1", 8)
    for x in (px, bad):
        x.close()
    echo.close()


def test_p2p_connection_through_proxy(core, node_factory, tmp_path):  # noqa: F811
    a, addr = node_factory(("-listen=1", "-port=0", "-listenonion=0"))
    client(a).generatetoaddress(3, addr)
    px = FakeSocks5()
    os.makedirs(tmp_path / "b", exist_ok=True)
    b, _ = node_factory((f"-proxy=127.0.0.1:{px.port}", f"-connect=127.0.0.1:{a.connman.port}",
                         f"-datadir={tmp_path / 'b'}"))
    cb = client(b)
    deadline = time.time() + 20
    while time.time() < deadline and cb.getblockcount() < 3:
        time.sleep(0.1)
    assert cb.getblockcount() == 3
    assert px.requests and px.requests[0][:2] == ("127.0.0.1", a.connman.port)
    nets = {n["name"]: n for n in cb.getnetworkinfo()["networks"]}
    assert nets["ipv4"]["proxy"] == f"127.0.0.1:{px.port}" and nets["ipv4"]["proxy_randomize_credentials"]
    px.close()
