"""Peer connections and headers-first block sync.

Parity (a deliberately small subset of SURVEY N1/N2; the reference's CConnman /
PeerLogicValidation are DEFER): CConnman listen/connect (src/net.cpp:2304-2420),
one reader thread per peer instead of the select() loop, and the message
handling of PeerLogicValidation::ProcessMessage (src/net_processing.cpp:1527)
for version / verack / ping / pong / getheaders / headers / inv / getdata / block /
sendheaders. Headers-first sync follows src/net_processing.cpp:1369-1500:
`getheaders` with a block locator, <= 2000 headers per reply, a follow-up
`getheaders` while replies are full, then `getdata` for the block bodies.

The MI355X difference is where a `headers` batch goes: instead of the reference's
serial CheckBlockHeader per header under cs_main (src/validation.cpp:12017-12035),
the whole batch is PoW-checked in bulk (models/verify.process_headers — GPU batch
kernels when the node has GPUs, all host cores otherwise), then DarkGravityWave and
the contextual rules run header by header on the C++ header chain.
"""
from __future__ import annotations

import socket
import struct
import threading
import time

from .. import core
from ..utils import log, sync
from ..utils.metrics import REGISTRY
from . import protocol as P

_core = core()
DEFAULT_MISBEHAVING_BANTIME = 60 * 60 * 24  # -bantime (src/net.h)


class Peer:
    def __init__(self, mgr: "ConnectionManager", sock: socket.socket, addr, inbound: bool):
        self.mgr, self.sock, self.addr, self.inbound = mgr, sock, addr, inbound
        self.id = mgr.next_id()
        self.info: dict = {}
        self.sent_version = False
        self.verack = False
        self.send_headers = False
        self.misbehavior = 0
        self.bytes_sent = self.bytes_recv = 0
        self.known_txs: set[bytes] = set()  # filterInventoryKnown
        self.fee_filter = 0
        self.connected_at = time.time()
        self.last_recv = self.last_send = 0.0
        self._send_lock = threading.Lock()
        self.closed = threading.Event()
        self.thread = threading.Thread(target=self._run, name=f"p2p-peer{self.id}", daemon=True)

    def send(self, cmd: str, payload: bytes = b"") -> None:
        msg = P.frame(self.mgr.magic, cmd, payload)
        with self._send_lock:
            self.sock.sendall(msg)
        self.bytes_sent += len(msg)
        self.mgr.total_sent += len(msg)
        self.last_send = time.time()
        REGISTRY.inc("p2p_bytes_sent_total", len(msg), command=cmd)

    def send_version(self) -> None:
        self.sent_version = True
        self.send("version", P.version_payload(self.mgr.state.height(), nonce=self.mgr.local_nonce))

    def misbehaving(self, score: int, why: str) -> None:
        """Misbehaving() / DoS ban score (src/net_processing.cpp): disconnect at 100."""
        self.misbehavior += score
        log.log_print("net", f"peer {self.id} misbehaving +{score} ({why}), total {self.misbehavior}")
        if self.misbehavior >= 100:
            self.mgr.ban(self.addr[0], DEFAULT_MISBEHAVING_BANTIME)
            self.close()

    def close(self) -> None:
        if not self.closed.is_set():
            self.closed.set()
            try:
                self.sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            self.sock.close()

    def _run(self) -> None:
        try:
            if not self.inbound:
                self.send_version()
            while not self.closed.is_set():
                cmd, payload = P.read_message(self.sock, self.mgr.magic)
                self.bytes_recv += P.HEADER_SIZE + len(payload)
                self.mgr.total_recv += P.HEADER_SIZE + len(payload)
                self.last_recv = time.time()
                REGISTRY.inc("p2p_bytes_recv_total", P.HEADER_SIZE + len(payload), command=cmd)
                self.mgr.handle(self, cmd, payload)
        except (ConnectionError, OSError, P.ProtocolError, struct.error, ValueError) as e:
            if not self.closed.is_set():
                log.log_print("net", f"peer {self.id} disconnected: {e}")
        finally:
            self.close()
            self.mgr.remove(self)

    @property
    def relay_txs(self) -> bool:
        return bool(self.info.get("relay", True))

    def as_dict(self) -> dict:
        host, port = self.addr[:2]
        return {"id": self.id, "addr": f"{host}:{port}", "inbound": self.inbound, "version": self.info.get("version", 0),
                "subver": self.info.get("user_agent", ""), "startingheight": self.info.get("start_height", -1),
                "bytessent": self.bytes_sent, "bytesrecv": self.bytes_recv, "conntime": int(self.connected_at),
                "lastsend": int(self.last_send), "lastrecv": int(self.last_recv), "banscore": self.misbehavior,
                "synced_headers": self.mgr.state.height(), "relaytxes": self.info.get("relay", True)}


class ConnectionManager:
    """Listener + outbound connections + message handling for one node."""

    def __init__(self, state, params, gpus: list[int] | None = None, listen: tuple[str, int] | None = None,
                 verify_mode: str = "auto"):
        self.state, self.params = state, params
        self.magic = bytes(params.message_start)
        self.gpus = gpus or None
        self.verify_mode = verify_mode
        self.listen_addr = listen
        self.local_nonce = int.from_bytes(struct.pack("<d", time.time()), "little") ^ id(self)
        self.peers: list[Peer] = []
        self._lock = sync.make_lock("cs_vNodes")
        self._id = 0
        self._server: socket.socket | None = None
        self._stop = threading.Event()
        self.port: int | None = None
        self.sync_lock = sync.make_lock("cs_headers")  # one headers batch is processed at a time
        self.total_sent = self.total_recv = 0
        self.started = time.time()
        self.network_active = True
        self.banned: dict[str, dict] = {}   # address -> {"banned_until", "ban_created", "ban_reason"}
        self.added_nodes: list[str] = []    # addnode "add" list (getaddednodeinfo)

    # ---------------------------------------------------------------- lifecycle
    def next_id(self) -> int:
        with self._lock:
            self._id += 1
            return self._id

    def start(self) -> None:
        if self.listen_addr is not None:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind(self.listen_addr)
            srv.listen(16)
            self._server = srv
            self.port = srv.getsockname()[1]
            threading.Thread(target=self._accept_loop, name="p2p-listen", daemon=True).start()
            log.log_printf(f"P2P listening on {self.listen_addr[0]}:{self.port}")

    def _accept_loop(self) -> None:
        while not self._stop.is_set():
            try:
                sock, addr = self._server.accept()
            except OSError:
                break
            if not self.network_active or self.is_banned(addr[0]):
                sock.close()  # CConnman::AcceptConnection drops banned / inactive-network peers
                continue
            self._add(sock, addr, inbound=True)

    def connect(self, host: str, port: int, timeout: float = 10.0) -> Peer:
        if not self.network_active:
            raise ConnectionError("network is disabled (setnetworkactive false)")
        sock = socket.create_connection((host, port), timeout=timeout)
        sock.settimeout(None)
        return self._add(sock, (host, port), inbound=False)

    def _add(self, sock, addr, inbound: bool) -> Peer:
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        p = Peer(self, sock, addr, inbound)
        with self._lock:
            self.peers.append(p)
        p.thread.start()
        return p

    def remove(self, p: Peer) -> None:
        with self._lock:
            if p in self.peers:
                self.peers.remove(p)

    def stop(self) -> None:
        self._stop.set()
        if self._server is not None:
            self._server.close()
        for p in list(self.peers):
            p.close()

    def peer_count(self) -> int:
        with self._lock:
            return sum(1 for p in self.peers if p.verack)

    # ---------------------------------------------------------------- bans / control (src/rpc/net.cpp)
    def ban(self, address: str, seconds: int, absolute: bool = False, reason: str = "node misbehaving") -> None:
        now = int(time.time())
        until = int(seconds) if absolute else now + int(seconds or DEFAULT_MISBEHAVING_BANTIME)
        self.banned[address] = {"address": address, "banned_until": until, "ban_created": now, "ban_reason": reason}
        for p in list(self.peers):
            if p.addr[0] == address:
                p.close()

    def unban(self, address: str) -> bool:
        return self.banned.pop(address, None) is not None

    def is_banned(self, address: str) -> bool:
        e = self.banned.get(address)
        if e is not None and e["banned_until"] < time.time():
            self.banned.pop(address, None)
            return False
        return e is not None

    def list_banned(self) -> list[dict]:
        for a in list(self.banned):
            self.is_banned(a)  # sweep expired entries
        return list(self.banned.values())

    def disconnect(self, address: str | None = None, node_id: int | None = None) -> bool:
        for p in list(self.peers):
            host, port = p.addr[:2]
            if (node_id is not None and p.id == node_id) or (address is not None and address in (f"{host}:{port}", host)):
                p.close()
                return True
        return False

    def set_network_active(self, active: bool) -> None:
        self.network_active = bool(active)
        if not active:
            for p in list(self.peers):
                p.close()

    # ---------------------------------------------------------------- relay
    def announce_block(self, header) -> None:
        """New tip: `headers` to peers that asked for sendheaders, `inv` to the rest."""
        act = self.params.kawpow_activation_time
        h = self.state.block_hash(header)
        for p in list(self.peers):
            if not p.verack:
                continue
            try:
                if p.send_headers:
                    p.send("headers", _core.headers_msg_encode([header], act))
                else:
                    p.send("inv", P.inv_payload([(P.MSG_BLOCK, h)]))
            except OSError:
                p.close()

    def announce_tx(self, txid: bytes, skip: "Peer | None" = None) -> None:
        """RelayTransaction: `inv` MSG_TX to every peer that has not sent us this tx."""
        for p in list(self.peers):
            if p is skip or not p.verack or not p.relay_txs or txid in p.known_txs:
                continue
            p.known_txs.add(txid)
            try:
                p.send("inv", P.inv_payload([(P.MSG_TX, txid)]))
            except OSError:
                p.close()

    # ---------------------------------------------------------------- message handling
    def handle(self, peer: Peer, cmd: str, p: bytes) -> None:
        fn = getattr(self, "on_" + cmd, None)
        if fn is None:
            return  # unknown / unsupported messages are ignored, as the reference does
        if cmd not in ("version",) and peer.info == {}:
            peer.misbehaving(1, f"{cmd} before version")
            return
        fn(peer, p)

    def on_version(self, peer: Peer, p: bytes) -> None:
        info = P.parse_version(p)
        if info["nonce"] == self.local_nonce:
            log.log_print("net", f"connected to self at {peer.addr}, disconnecting")
            peer.close()
            return
        if info["version"] < P.MIN_PEER_PROTO_VERSION:
            log.log_print("net", f"peer {peer.id} using obsolete version {info['version']}; disconnecting")
            peer.close()
            return
        peer.info = info
        if peer.inbound and not peer.sent_version:
            peer.send_version()
        peer.send("verack")

    def on_verack(self, peer: Peer, p: bytes) -> None:
        peer.verack = True
        peer.send("sendheaders")
        self.request_headers(peer)

    def on_sendheaders(self, peer: Peer, p: bytes) -> None:
        peer.send_headers = True

    def on_ping(self, peer: Peer, p: bytes) -> None:
        peer.send("pong", p[:8])

    def on_pong(self, peer: Peer, p: bytes) -> None:
        pass

    def request_headers(self, peer: Peer) -> None:
        peer.send("getheaders", P.getheaders_payload(P.locator(self.state.chain)))

    def on_getheaders(self, peer: Peer, p: bytes) -> None:
        loc, stop = P.parse_getheaders(p)
        chain = self.state.chain
        start = 0
        for h in loc:  # first locator entry on our active chain = fork point
            idx = chain.find(h)
            if idx is not None and chain.in_active_chain(idx):
                start = idx.height + 1
                break
        out = []
        for height in range(start, min(chain.height(), start + P.MAX_HEADERS_RESULTS - 1) + 1):
            idx = chain.at_height(height)
            out.append(idx.header)
            if idx.hash == stop:
                break
        peer.send("headers", _core.headers_msg_encode(out, self.params.kawpow_activation_time))

    def on_headers(self, peer: Peer, p: bytes) -> None:
        from ..models.verify import process_headers

        headers = _core.headers_msg_decode(p, self.params.kawpow_activation_time)
        if not headers:
            return
        with self.sync_lock:
            chain = self.state.chain
            if chain.find(headers[0].prev) is None:  # unconnecting headers: ask from our locator
                self.request_headers(peer)
                return
            self.state.arm_reorg_guard(self.peer_count())
            t0 = time.perf_counter()
            res = process_headers(chain, headers, self.state.adjusted_time(), gpus=self.gpus, mode=self.verify_mode)
            REGISTRY.inc("p2p_headers_accepted_total", res["accepted"])
            REGISTRY.set("p2p_headers_batch_seconds", time.perf_counter() - t0)
            log.log_print("net", f"peer {peer.id}: {res['accepted']}/{len(headers)} headers accepted "
                                 f"(pow {res['pow_s'] * 1e3:.1f} ms, context {res['context_s'] * 1e3:.1f} ms)")
            if res["reject"] is not None:
                peer.misbehaving(100 if res["reject"]["reason"] in ("high-hash", "invalid-mix-hash", "bad-diffbits")
                                 else 20, f"invalid header: {res['reject']}")
                return
        want = [self.state.block_hash(h) for h in headers]
        want = [h for h in want if h not in self.state.block_pos]
        for k in range(0, len(want), 128):
            peer.send("getdata", P.inv_payload([(P.MSG_BLOCK | P.MSG_WITNESS_FLAG, h) for h in want[k:k + 128]]))
        if len(headers) == P.MAX_HEADERS_RESULTS:
            self.request_headers(peer)

    def on_inv(self, peer: Peer, p: bytes) -> None:
        items = P.parse_inv(p)
        if len(items) > P.MAX_INV_SZ:
            peer.misbehaving(20, "oversized inv")
            return
        if any(t & ~P.MSG_WITNESS_FLAG == P.MSG_BLOCK and self.state.chain.find(h) is None for t, h in items):
            self.request_headers(peer)
        want = []
        for t, h in items:
            if t & ~P.MSG_WITNESS_FLAG == P.MSG_TX:
                peer.known_txs.add(h)
                if h not in self.state.mempool:
                    want.append((P.MSG_TX | P.MSG_WITNESS_FLAG, h))
        if want:
            peer.send("getdata", P.inv_payload(want))

    def on_tx(self, peer: Peer, p: bytes) -> None:
        """AcceptToMemoryPool for a relayed tx (UTXO set, scripts, fees); accepted transactions
        are relayed to the other peers by the mempool signal."""
        tx = _core.Transaction.deserialize(p)
        txid = tx.txid()
        peer.known_txs.add(txid)
        REGISTRY.inc("p2p_tx_received_total", 1)
        if txid in self.state.mempool:
            return
        ok, reason, _ = self.state.accept_to_mempool(tx)
        if not ok:
            REGISTRY.inc("p2p_tx_rejected_total", 1)
            log.log_print("mempool", f"tx {_core.u256_hex(txid)} from peer {peer.id} rejected: {reason}")

    def on_mempool(self, peer: Peer, p: bytes) -> None:
        """BIP35: inv of every pool txid (in MAX_INV_SZ chunks)."""
        ids = list(self.state.mempool)
        peer.known_txs.update(ids)
        for k in range(0, len(ids), P.MAX_INV_SZ):
            peer.send("inv", P.inv_payload([(P.MSG_TX, h) for h in ids[k:k + P.MAX_INV_SZ]]))

    def on_feefilter(self, peer: Peer, p: bytes) -> None:
        (peer.fee_filter,) = struct.unpack_from("<q", p, 0)

    def on_getdata(self, peer: Peer, p: bytes) -> None:
        missing = []
        for t, h in P.parse_inv(p):
            if t & ~P.MSG_WITNESS_FLAG == P.MSG_BLOCK:
                raw = self.state.get_block_raw(h)
                if raw is None:
                    missing.append((t, h))
                else:
                    peer.send("block", raw)
            elif t & ~P.MSG_WITNESS_FLAG == P.MSG_TX and h in self.state.mempool:
                peer.send("tx", self.state.mempool[h].tx.serialize(bool(t & P.MSG_WITNESS_FLAG)))
            else:
                missing.append((t, h))
        if missing:
            peer.send("notfound", P.inv_payload(missing))

    def on_block(self, peer: Peer, p: bytes) -> None:
        blk = _core.Block.deserialize(p, self.params.kawpow_activation_time)
        self.state.arm_reorg_guard(self.peer_count())
        st = self.state.process_new_block(blk)
        REGISTRY.inc("p2p_blocks_received_total", 1, ok=st.ok)
        if not st.ok and st.reject != "duplicate":
            peer.misbehaving(st.dos or 0, f"invalid block: {st.reject}")
