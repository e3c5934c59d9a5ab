"""Proxy-aware outbound connections: SOCKS5 and per-network proxies.

Parity (behaviour): src/netbase.cpp — `Socks5()` (RFC 1928 CONNECT by domain name, with the
RFC 1929 username/password step used by -proxyrandomize), `ConnectThroughProxy`, `SetProxy` /
`GetProxy` / `IsProxy` per network, and the option handling of src/init.cpp (`-proxy`,
`-onion` / `-noonion`, `-proxyrandomize`, `-onlynet`). Network classes follow
CNetAddr::GetNetwork: `.onion` names are NET_TOR, literal IPv6 is NET_IPV6, the rest NET_IPV4.
"""
from __future__ import annotations

import ipaddress
import os
import socket
import struct
import threading
from dataclasses import dataclass

NETWORKS = ("ipv4", "ipv6", "onion")

# Socks5 reply codes (src/netbase.cpp: SOCKS5Reply) -> the reference's error strings
_SOCKS5_ERRORS = {
    0x01: "general failure", 0x02: "connection not allowed", 0x03: "network unreachable",
    0x04: "host unreachable", 0x05: "connection refused", 0x06: "TTL expired",
    0x07: "protocol error", 0x08: "address type not supported",
}


class ProxyError(ConnectionError):
    pass


@dataclass(frozen=True)
class Proxy:
    """proxyType: where the SOCKS5 server is and whether each connection gets fresh
    credentials (-proxyrandomize: Tor then isolates every stream on its own circuit)."""
    host: str
    port: int
    randomize_credentials: bool = True

    def __str__(self) -> str:
        return f"[{self.host}]:{self.port}" if ":" in self.host else f"{self.host}:{self.port}"


def parse_host_port(s: str, default_port: int) -> tuple[str, int]:
    """SplitHostPort: "host", "host:port", "[v6]:port", bare IPv6."""
    s = s.strip()
    if s.startswith("["):
        host, _, rest = s[1:].partition("]")
        return host, int(rest[1:]) if rest.startswith(":") else default_port
    if s.count(":") == 1:
        host, port = s.split(":")
        return host, int(port)
    return s, default_port


def network_of(host: str) -> str:
    if host.lower().endswith(".onion"):
        return "onion"
    try:
        return "ipv6" if ipaddress.ip_address(host).version == 6 else "ipv4"
    except ValueError:
        return "ipv4"  # a name: resolved over IPv4 (or by the proxy)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    out = b""
    while len(out) < n:
        chunk = sock.recv(n - len(out))
        if not chunk:
            raise ProxyError("Error reading proxy response")
        out += chunk
    return out


def socks5_handshake(sock: socket.socket, dest: str, port: int, auth: tuple[str, str] | None = None) -> None:
    """Socks5(): greeting (no-auth, plus user/pass when `auth`), optional RFC 1929 login, then
    CONNECT to `dest` as a domain name (the proxy resolves it; .onion names need Tor)."""
    if len(dest) > 255:
        raise ProxyError("Hostname too long")
    sock.sendall(b"\x05\x02\x00\x02" if auth else b"\x05\x01\x00")
    ver, method = _recv_exact(sock, 2)
    if ver != 0x05:
        raise ProxyError("Proxy failed to initialize")
    if method == 0x02 and auth:
        user, pw = (x.encode() for x in auth)
        if len(user) > 255 or len(pw) > 255:
            raise ProxyError("Proxy username or password too long")
        sock.sendall(bytes([0x01, len(user)]) + user + bytes([len(pw)]) + pw)
        aver, status = _recv_exact(sock, 2)
        if aver != 0x01 or status != 0x00:
            raise ProxyError("Proxy authentication unsuccessful")
    elif method != 0x00:
        raise ProxyError("Proxy requested wrong authentication method %02x" % method)
    host = dest.encode()
    sock.sendall(b"\x05\x01\x00\x03" + bytes([len(host)]) + host + struct.pack(">H", port))
    ver, rep, rsv, atyp = _recv_exact(sock, 4)
    if ver != 0x05:
        raise ProxyError("Proxy failed to accept request")
    if rep != 0x00:
        raise ProxyError(f"Proxy error: {_SOCKS5_ERRORS.get(rep, 'unknown')}")
    if rsv != 0x00:
        raise ProxyError("Error: malformed proxy response")
    if atyp == 0x01:
        _recv_exact(sock, 4)
    elif atyp == 0x04:
        _recv_exact(sock, 16)
    elif atyp == 0x03:
        _recv_exact(sock, _recv_exact(sock, 1)[0])
    else:
        raise ProxyError("Error: malformed proxy response")
    _recv_exact(sock, 2)  # bound port


class ProxyTable:
    """SetProxy / GetProxy / SetNameProxy and the reachability of each network
    (SetLimited / IsLimited), shared by every outbound connection of one node."""

    def __init__(self):
        self._lock = threading.Lock()
        self.proxies: dict[str, Proxy] = {}
        self.limited: set[str] = set()
        self._counter = 0

    def set_proxy(self, net: str, proxy: Proxy | None) -> None:
        with self._lock:
            if proxy is None:
                self.proxies.pop(net, None)
            else:
                self.proxies[net] = proxy

    def get_proxy(self, net: str) -> Proxy | None:
        with self._lock:
            return self.proxies.get(net)

    def set_limited(self, net: str, limited: bool = True) -> None:
        with self._lock:
            (self.limited.add if limited else self.limited.discard)(net)

    def is_reachable(self, net: str) -> bool:
        with self._lock:
            if net in self.limited:
                return False
            return net != "onion" or "onion" in self.proxies

    def configure(self, args) -> None:
        """init.cpp step 3: -onlynet limits the other networks; -proxy serves IPv4, IPv6 and
        (unless -onion says otherwise) onion; -onion=host:port or -noonion for NET_TOR."""
        only = [n.lower() for n in args.get_list("onlynet")]
        if only:
            for n in NETWORKS:
                self.set_limited(n, n not in only)
        randomize = args.get_bool("proxyrandomize", True)
        proxy_arg = args.get("proxy")
        if proxy_arg and proxy_arg != "0":
            host, port = parse_host_port(proxy_arg, 9050)
            p = Proxy(host, port, randomize)
            self.set_proxy("ipv4", p)
            self.set_proxy("ipv6", p)
            self.set_proxy("onion", p)
        onion_arg = args.get("onion")
        if onion_arg is not None:
            if onion_arg in ("0", ""):
                self.set_proxy("onion", None)
                self.set_limited("onion")
            else:
                host, port = parse_host_port(onion_arg, 9050)
                self.set_proxy("onion", Proxy(host, port, randomize))
                self.set_limited("onion", False)

    def credentials(self) -> tuple[str, str]:
        """-proxyrandomize: a fresh user/password per connection (the reference's counter
        string), so Tor's IsolateSOCKSAuth puts each stream on its own circuit."""
        with self._lock:
            self._counter += 1
            tag = f"{os.getpid()}-{self._counter}"
        return tag, tag

    def connect(self, host: str, port: int, timeout: float = 10.0) -> socket.socket:
        """ConnectNode's socket step: direct TCP, or through the network's proxy."""
        net = network_of(host)
        if not self.is_reachable(net):
            raise ConnectionError(f"network {net} is not reachable (-onlynet / no onion proxy)")
        proxy = self.get_proxy(net)
        if proxy is None:
            return socket.create_connection((host, port), timeout=timeout)
        sock = socket.create_connection((proxy.host, proxy.port), timeout=timeout)
        try:
            socks5_handshake(sock, host, port, self.credentials() if proxy.randomize_credentials else None)
        except Exception:
            sock.close()
            raise
        return sock

    def describe(self) -> list[dict]:
        """getnetworkinfo "networks" entries (GetNetworksInfo, src/rpc/net.cpp)."""
        out = []
        for n in NETWORKS:
            p = self.get_proxy(n)
            out.append({"name": n, "limited": n in self.limited, "reachable": self.is_reachable(n),
                        "proxy": str(p) if p else "",
                        "proxy_randomize_credentials": bool(p and p.randomize_credentials)})
        return out
