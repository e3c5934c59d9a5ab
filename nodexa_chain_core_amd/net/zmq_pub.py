"""ZMQ block/tx notifications over a self-contained ZMTP 3.0 PUB endpoint.

Parity: CZMQNotificationInterface + CZMQPublish*Notifier (src/zmq/
zmqnotificationinterface.cpp:41-45, src/zmq/zmqpublishnotifier.cpp:25,136-143):
`-zmqpubhashblock=tcp://host:port`, `-zmqpubrawblock=...`, `-zmqpubhashtx=...`,
`-zmqpubrawtx=...`, `-zmqpubrawmessage=...` (asset messages as the reference's JSON string);
every notification is a 3-frame multipart message
[topic][payload][little-endian u32 sequence number], one sequence counter per
topic; block/tx hashes are sent in display (reversed) byte order as the
reference does. libzmq is not available in this environment, so the endpoint
speaks the wire protocol itself (ZMTP 3.0/3.1, NULL mechanism): the 64-byte
greeting, READY with Socket-Type=PUB, and subscription prefixes sent by SUB
peers either as 0x01-prefixed messages (3.0) or SUBSCRIBE commands (3.1). Any
libzmq SUB socket can subscribe to it.
"""
from __future__ import annotations

import socket
import struct
import threading

from ..utils import log

TOPICS = ("hashblock", "hashtx", "rawblock", "rawtx", "rawmessage")


def greeting(as_server: bool = True) -> bytes:
    return (b"\xff" + b"\0" * 8 + b"\x7f" + bytes([3, 0]) + b"NULL".ljust(20, b"\0") + bytes([1 if as_server else 0])
            + b"\0" * 31)


def frame(body: bytes, more: bool = False, command: bool = False) -> bytes:
    flags = (1 if more else 0) | (4 if command else 0)
    if len(body) > 255:
        return bytes([flags | 2]) + struct.pack(">Q", len(body)) + body
    return bytes([flags, len(body)]) + body


def ready_command(socket_type: str) -> bytes:
    props = b"\x0bSocket-Type" + struct.pack(">I", len(socket_type)) + socket_type.encode()
    return frame(b"\x05READY" + props, command=True)


def read_frame(sock: socket.socket) -> tuple[int, bytes]:
    def exact(n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            c = sock.recv(n - len(buf))
            if not c:
                raise ConnectionError("zmq peer closed")
            buf += c
        return bytes(buf)

    flags = exact(1)[0]
    size = struct.unpack(">Q", exact(8))[0] if flags & 2 else exact(1)[0]
    return flags, exact(size) if size else b""


class _Sub:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.prefixes: set[bytes] = set()
        self.lock = threading.Lock()
        self.alive = True


class ZmqPublisher:
    """One bound PUB endpoint; `publish(topic, payload)` fans out to matching subscribers."""

    def __init__(self, host: str, port: int):
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind((host, port))
        self.srv.listen(16)
        self.port = self.srv.getsockname()[1]
        self.subs: list[_Sub] = []
        self.seq: dict[str, int] = {}
        self._lock = threading.Lock()
        self._stop = threading.Event()
        threading.Thread(target=self._accept, name="zmq-pub", daemon=True).start()

    def _accept(self) -> None:
        while not self._stop.is_set():
            try:
                s, _ = self.srv.accept()
            except OSError:
                break
            threading.Thread(target=self._serve, args=(s,), name="zmq-sub", daemon=True).start()

    def _serve(self, s: socket.socket) -> None:
        sub = _Sub(s)
        try:
            s.sendall(greeting())
            peer = b""
            while len(peer) < 64:
                c = s.recv(64 - len(peer))
                if not c:
                    return
                peer += c
            if peer[0] != 0xFF or peer[9] != 0x7F or peer[10] < 3:
                return
            s.sendall(ready_command("PUB"))
            with self._lock:
                self.subs.append(sub)
            while True:
                flags, body = read_frame(s)
                if flags & 4:  # command frame
                    name_len = body[0] if body else 0
                    name = body[1:1 + name_len]
                    if name == b"SUBSCRIBE":
                        sub.prefixes.add(body[1 + name_len:])
                    elif name == b"CANCEL":
                        sub.prefixes.discard(body[1 + name_len:])
                elif body[:1] == b"\x01":
                    sub.prefixes.add(body[1:])
                elif body[:1] == b"\x00":
                    sub.prefixes.discard(body[1:])
        except (ConnectionError, OSError, IndexError, struct.error):
            pass
        finally:
            sub.alive = False
            with self._lock:
                if sub in self.subs:
                    self.subs.remove(sub)
            s.close()

    def publish(self, topic: str, payload: bytes) -> None:
        with self._lock:
            seq = self.seq.get(topic, 0)
            self.seq[topic] = seq + 1
            subs = list(self.subs)
        t = topic.encode()
        msg = frame(t, more=True) + frame(payload, more=True) + frame(struct.pack("<I", seq))
        for sub in subs:
            if any(t.startswith(p) for p in sub.prefixes):
                try:
                    with sub.lock:
                        sub.sock.sendall(msg)
                except OSError:
                    sub.alive = False

    def stop(self) -> None:
        self._stop.set()
        self.srv.close()
        for sub in list(self.subs):
            try:
                sub.sock.close()
            except OSError:
                pass


class ZmqNotifier:
    """Validation-interface subscriber that publishes the enabled topics (-zmqpub<topic>=tcp://host:port)."""

    def __init__(self, state, endpoints: dict[str, str]):
        self.state = state
        self.pubs: dict[str, ZmqPublisher] = {}
        by_ep: dict[str, ZmqPublisher] = {}
        for topic, ep in endpoints.items():
            if topic not in TOPICS:
                raise ValueError(f"unknown zmq topic {topic}")
            if ep not in by_ep:
                if not ep.startswith("tcp://"):
                    raise ValueError(f"zmq endpoint must be tcp://host:port, got {ep}")
                host, _, port = ep[6:].rpartition(":")
                by_ep[ep] = ZmqPublisher(host or "127.0.0.1", int(port))
                log.log_print("zmq", f"zmq{topic} bound to tcp://{host}:{by_ep[ep].port}")
            self.pubs[topic] = by_ep[ep]

    def block_connected(self, block, index) -> None:
        if "hashblock" in self.pubs:
            self.pubs["hashblock"].publish("hashblock", bytes(index.hash)[::-1])
        if "rawblock" in self.pubs:
            self.pubs["rawblock"].publish("rawblock", block.serialize(self.state.params.kawpow_activation_time))
        for tx in block.vtx:
            if "hashtx" in self.pubs:
                self.pubs["hashtx"].publish("hashtx", bytes(tx.txid())[::-1])
            if "rawtx" in self.pubs:
                self.pubs["rawtx"].publish("rawtx", tx.serialize(True))

    # the other ValidationInterface hooks are not used
    def transaction_added_to_mempool(self, tx) -> None:  # CZMQNotificationInterface::TransactionAddedToMempool
        if "hashtx" in self.pubs:
            self.pubs["hashtx"].publish("hashtx", bytes(tx.txid())[::-1])
        if "rawtx" in self.pubs:
            self.pubs["rawtx"].publish("rawtx", tx.serialize(True))

    def new_asset_message(self, message) -> None:  # CZMQPublishNewAssetMessageNotifier ("rawmessage")
        if "rawmessage" in self.pubs:
            self.pubs["rawmessage"].publish("rawmessage", message.zmq_json().encode())

    def updated_block_tip(self, *a) -> None: ...

    def block_checked(self, *a) -> None: ...

    def block_found(self, *a) -> None: ...

    def stop(self) -> None:
        for p in set(self.pubs.values()):
            p.stop()
