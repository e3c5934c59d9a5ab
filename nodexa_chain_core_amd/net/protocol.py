"""P2P wire protocol: message framing and the payloads headers-first sync needs.

Parity: CMessageHeader (src/protocol.h:34-41: 4-byte network magic, 12-byte
NUL-padded command, u32 payload size, first 4 bytes of SHA256d(payload)),
NetMsgType names (src/protocol.h:79-266), PROTOCOL_VERSION 70028 and the
KawPow / X16RV2 minimum versions (src/version.h:13-33), the `version` payload
(src/net_processing.cpp:301-302), block locators (src/chain.cpp GetLocator),
`getheaders` / `headers` (<= MAX_HEADERS_RESULTS = 2000, src/validation.h:105)
and `inv` / `getdata` entries (src/protocol.h CInv; MSG_BLOCK = 2,
MSG_WITNESS_FLAG = 1 << 30). Header payloads are encoded/decoded natively
(_core.headers_msg_encode / headers_msg_decode) in the 80 / 120-byte formats
gated by the KawPow activation time.
"""
from __future__ import annotations

import os
import socket
import struct
import time

from .. import core

_core = core()

PROTOCOL_VERSION = 70028
KAWPOW_VERSION = 70027
MIN_PEER_PROTO_VERSION = 70025  # X16RV2_VERSION
NODE_NETWORK = 1
NODE_WITNESS = 1 << 3
NODE_BLOOM = 1 << 2    # BIP111: bloom filters served (-peerbloomfilters)
MAX_HEADERS_RESULTS = 2000
MAX_MESSAGE_SIZE = 32 * 1024 * 1024  # MAX_PROTOCOL_MESSAGE_LENGTH after the HIP2 block-size change
MSG_TX, MSG_BLOCK = 1, 2
MAX_INV_SZ = 50000  # src/net_processing.h
MSG_WITNESS_FLAG = 1 << 30
HEADER_SIZE = 24
USER_AGENT = "/nodexa-mi355x:0.1.0/"

COMMANDS = ("version", "verack", "addr", "inv", "getdata", "merkleblock", "getblocks", "getheaders", "tx",
            "headers", "block", "getaddr", "mempool", "ping", "pong", "notfound", "filterload", "filteradd",
            "filterclear", "reject", "sendheaders", "feefilter", "sendcmpct", "cmpctblock", "getblocktxn",
            "blocktxn")


class ProtocolError(Exception):
    pass


def checksum(payload: bytes) -> bytes:
    return _core.sha256d(payload)[:4]


def frame(magic: bytes, command: str, payload: bytes = b"") -> bytes:
    if len(command) > 12:
        raise ValueError("command longer than 12 bytes")
    return magic + command.encode().ljust(12, b"\0") + struct.pack("<I", len(payload)) + checksum(payload) + payload


def parse_header(magic: bytes, hdr: bytes) -> tuple[str, int, bytes]:
    if len(hdr) != HEADER_SIZE:
        raise ProtocolError("short message header")
    if hdr[:4] != magic:
        raise ProtocolError(f"bad network magic {hdr[:4].hex()}")
    raw = hdr[4:16]
    cmd = raw.rstrip(b"\0")
    if b"\0" in cmd or not all(0x20 < c < 0x7f for c in cmd):
        raise ProtocolError("malformed command")
    (size,) = struct.unpack("<I", hdr[16:20])
    if size > MAX_MESSAGE_SIZE:
        raise ProtocolError(f"oversized message ({size} bytes)")
    return cmd.decode(), size, hdr[20:24]


def recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed the connection")
        buf += chunk
    return bytes(buf)


def read_message(sock: socket.socket, magic: bytes) -> tuple[str, bytes]:
    cmd, size, chk = parse_header(magic, recv_exact(sock, HEADER_SIZE))
    payload = recv_exact(sock, size) if size else b""
    if checksum(payload) != chk:
        raise ProtocolError(f"bad checksum on {cmd}")
    return cmd, payload


# ---------------------------------------------------------------- compact size / var str
def ser_compact(n: int) -> bytes:
    if n < 253:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + struct.pack("<H", n)
    if n <= 0xFFFFFFFF:
        return b"\xfe" + struct.pack("<I", n)
    return b"\xff" + struct.pack("<Q", n)


def de_compact(b: bytes, off: int) -> tuple[int, int]:
    c = b[off]
    if c < 253:
        return c, off + 1
    if c == 253:
        return struct.unpack_from("<H", b, off + 1)[0], off + 3
    if c == 254:
        return struct.unpack_from("<I", b, off + 1)[0], off + 5
    return struct.unpack_from("<Q", b, off + 1)[0], off + 9


def ser_str(s: bytes) -> bytes:
    return ser_compact(len(s)) + s


def de_str(b: bytes, off: int) -> tuple[bytes, int]:
    n, off = de_compact(b, off)
    return b[off:off + n], off + n


# ---------------------------------------------------------------- payloads
def ser_netaddr(services: int, ip: str = "127.0.0.1", port: int = 0) -> bytes:
    ipv6 = b"\0" * 10 + b"\xff\xff" + socket.inet_aton(ip)
    return struct.pack("<Q", services) + ipv6 + struct.pack(">H", port)


def user_agent(comments: list[str] | None = None) -> str:
    """FormatSubVersion: /name:version(comment; comment)/ with -uacomment entries."""
    if not comments:
        return USER_AGENT
    return USER_AGENT[:-1] + "(" + "; ".join(comments) + ")/"


def version_payload(start_height: int, nonce: int | None = None, services: int = NODE_NETWORK | NODE_WITNESS,
                    relay: bool = True, their: tuple[str, int] = ("127.0.0.1", 0), agent: str = USER_AGENT) -> bytes:
    nonce = int.from_bytes(os.urandom(8), "little") if nonce is None else nonce
    return (struct.pack("<iQq", PROTOCOL_VERSION, services, int(time.time())) + ser_netaddr(services, *their) +
            ser_netaddr(services) + struct.pack("<Q", nonce) + ser_str(agent.encode()) +
            struct.pack("<i?", start_height, relay))


def parse_version(p: bytes) -> dict:
    version, services, t = struct.unpack_from("<iQq", p, 0)
    off = 20 + 26 + 26
    (nonce,) = struct.unpack_from("<Q", p, off)
    ua, off = de_str(p, off + 8)
    (height,) = struct.unpack_from("<i", p, off)
    relay = p[off + 4] != 0 if len(p) > off + 4 else True
    return {"version": version, "services": services, "time": t, "nonce": nonce, "user_agent": ua.decode(errors="replace"),
            "start_height": height, "relay": relay}


def locator(chain) -> list[bytes]:
    """CChain::GetLocator: the tip, 10 predecessors one by one, then exponentially sparser, genesis."""
    out, step = [], 1
    h = chain.height()
    while h > 0:
        out.append(chain.at_height(h).hash)
        if len(out) >= 10:
            step *= 2
        h -= step
    out.append(chain.at_height(0).hash)
    return out


def getheaders_payload(loc: list[bytes], stop: bytes = bytes(32)) -> bytes:
    return struct.pack("<I", PROTOCOL_VERSION) + ser_compact(len(loc)) + b"".join(loc) + stop


def parse_getheaders(p: bytes) -> tuple[list[bytes], bytes]:
    n, off = de_compact(p, 4)
    loc = [p[off + 32 * i: off + 32 * (i + 1)] for i in range(n)]
    off += 32 * n
    return loc, p[off:off + 32]


def inv_payload(items: list[tuple[int, bytes]]) -> bytes:
    return ser_compact(len(items)) + b"".join(struct.pack("<I", t) + h for t, h in items)


def parse_inv(p: bytes) -> list[tuple[int, bytes]]:
    n, off = de_compact(p, 0)
    out = []
    for _ in range(n):
        (t,) = struct.unpack_from("<I", p, off)
        out.append((t, p[off + 4: off + 36]))
        off += 36
    return out
