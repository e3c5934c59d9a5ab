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
the whole batch is PoW-checked in bulk, then DarkGravityWave and the contextual rules run on
the C++ header chain. With a GPU whose epoch DAGs are resident (a mining node), or with
`-p2pverifymode=dag`, the batch takes the device-resident path (models/verify.
process_batch_resident: one upload, PoW + block hashes + nBits on the GPU, one download, the bulk
insert); otherwise models/verify.process_headers (GPU light-mode kernels, or all host cores).
"""
from __future__ import annotations

import collections
import ipaddress
import os
import random
import socket
import struct
import threading
import time

from .. import core
from ..utils import log, sync
from ..utils.metrics import REGISTRY
from . import protocol as P
from .addrman import AddrMan, load_banlist, save_banlist
from .bloom import MAX_SCRIPT_ELEMENT_SIZE, BloomFilter, merkle_block
from .compact import (CompactBlock, blocktxn_payload, getblocktxn_payload, parse_blocktxn, parse_getblocktxn)
from .netbase import ProxyTable
from .timedata import TimeData

_core = core()
DEFAULT_MISBEHAVING_BANTIME = 60 * 60 * 24  # -bantime (src/net.h)
MSG_FILTERED_BLOCK, MSG_CMPCT_BLOCK = 3, 4
MAX_ADDR_TO_SEND = 1000
DEFAULT_MAX_OUTBOUND = 8  # MAX_OUTBOUND_CONNECTIONS


def _ser_addr(entries) -> bytes:
    """addr payload: (time u32, services u64, IPv6-mapped address, big-endian port) per entry."""
    out = P.ser_compact(len(entries))
    for ip, port, services, t in entries:
        a = ipaddress.ip_address(ip)
        raw = (b"\0" * 10 + b"\xff\xff" + a.packed) if a.version == 4 else a.packed
        out += struct.pack("<IQ", int(t) & 0xFFFFFFFF, services) + raw + struct.pack(">H", port)
    return out


def _parse_addr(p: bytes) -> list[tuple[str, int, int, int]]:
    n, off = P.de_compact(p, 0)
    out = []
    for _ in range(n):
        t, services = struct.unpack_from("<IQ", p, off)
        raw = p[off + 12:off + 28]
        (port,) = struct.unpack_from(">H", p, off + 28)
        off += 30
        a = ipaddress.ip_address(raw)
        ip = str(a.ipv4_mapped) if a.ipv4_mapped else str(a)
        out.append((ip, port, services, t))
    return out


DEFAULT_MAX_ORPHAN_TRANSACTIONS = 100   # -maxorphantx (src/net_processing.h)
ORPHAN_TX_EXPIRE_TIME = 20 * 60           # seconds (src/net_processing.cpp)
MAX_ORPHAN_TX_WEIGHT = 400_000            # MAX_STANDARD_TX_WEIGHT


class Peer:
    def __init__(self, mgr: "ConnectionManager", sock: socket.socket, addr, inbound: bool):
        self.mgr, self.sock, self.addr, self.inbound = mgr, sock, addr, inbound
        self.whitebind = False  # accepted on a -whitebind socket
        self.id = mgr.next_id()
        self.info: dict = {}
        self.sent_version = False
        self.verack = False
        self.send_headers = False
        self.misbehavior = 0
        self.bytes_sent = self.bytes_recv = 0
        self.known_txs: set[bytes] = set()  # filterInventoryKnown
        self.fee_filter = 0
        self.bloom: BloomFilter | None = None   # BIP37 filterload
        self.cmpct_version = 0                   # BIP152 sendcmpct version (0 = none)
        self.cmpct_hb = False                    # high-bandwidth mode: push cmpctblock unasked
        self.partial: dict[bytes, tuple] = {}    # block hash -> (CompactBlock, slots) awaiting blocktxn
        self.getaddr_answered = False
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
        self.mgr.record_sent(len(msg))
        self.last_send = time.time()
        REGISTRY.inc("p2p_bytes_sent_total", len(msg), command=cmd)

    def send_version(self) -> None:
        self.sent_version = True
        m = self.mgr
        self.send("version", P.version_payload(m.state.height(), nonce=m.local_nonce, services=m.local_services,
                                               relay=not m.blocks_only, agent=m.user_agent))

    @property
    def whitelisted(self) -> bool:
        """-whitelist: peers from these subnets are never banned and keep tx relay (-whitelistrelay)."""
        return self.whitebind or self.mgr.is_whitelisted(self.addr[0])

    def misbehaving(self, score: int, why: str) -> None:
        """Misbehaving() / DoS ban score (src/net_processing.cpp): disconnect at 100."""
        self.misbehavior += score
        log.log_print("net", f"peer {self.id} misbehaving +{score} ({why}), total {self.misbehavior}")
        if self.misbehavior >= 100 and self.whitelisted:
            log.log_printf(f"Warning: not punishing whitelisted peer {self.addr[0]}!")
        elif self.misbehavior >= 100:
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
                if self.mgr.drop_messages_test and random.randrange(self.mgr.drop_messages_test) == 0:
                    # -dropmessagestest=<n> (src/net_processing.cpp:1530)
                    log.log_printf("dropmessagestest DROPPING RECV MESSAGE")
                    continue
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
                "synced_headers": self.mgr.state.height(), "relaytxes": self.info.get("relay", True),
                "services": "%016x" % self.info.get("services", 0), "whitelisted": self.whitelisted,
                "timeoffset": self.info.get("timeoffset", 0)}


class ConnectionManager:
    """Listener + outbound connections + message handling for one node."""

    def __init__(self, state, params, gpus: list[int] | None = None, listen: tuple[str, int] | None = None,
                 verify_mode: str = "auto", datadir: str | None = None, connect_only: bool = False,
                 max_outbound: int = DEFAULT_MAX_OUTBOUND):
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
        # further listening sockets: (host, port, whitelisted) for extra -bind / -whitebind
        # addresses; peers accepted on a -whitebind socket are whitelisted whatever their address
        self.extra_binds: list[tuple[str, int, bool]] = []
        self._extra_servers: list[socket.socket] = []
        # -maxreceivebuffer / -maxsendbuffer (x1000 bytes per connection, src/net.h): each peer is
        # read and answered by its own thread, so a peer's only queues are its socket buffers;
        # they are sized to these bounds
        self.max_receive_buffer = 5000 * 1000
        self.max_send_buffer = 1000 * 1000
        self.drop_messages_test = 0  # -dropmessagestest=<n>: drop 1 in n received messages
        # vExtraTxnForCompact: orphans, rejected and replaced transactions kept for compact-block
        # reconstruction (-blockreconstructionextratxn, DEFAULT_BLOCK_RECONSTRUCTION_EXTRA_TXN)
        self.extra_txn: collections.deque = collections.deque(maxlen=100)
        self.allow_dns = True        # -dns: resolve names given to -addnode / -seednode / -connect
        self._stop = threading.Event()
        self.port: int | None = None
        self.sync_lock = sync.make_lock("cs_headers")  # one headers batch is processed at a time
        self.total_sent = self.total_recv = 0
        self.started = time.time()
        self.network_active = True
        self.banned: dict[str, dict] = {}   # address -> {"banned_until", "ban_created", "ban_reason"}
        self.added_nodes: list[str] = []    # addnode "add" list (getaddednodeinfo)
        # peer addresses (peers.dat) and bans (banlist.dat), CConnman's addrman / CBanDB
        self.datadir = datadir
        self.addrman = AddrMan(os.path.join(datadir, "peers.dat") if datadir else None)
        self.banlist_path = os.path.join(datadir, "banlist.dat") if datadir else None
        if self.banlist_path:
            self.banned.update(load_banlist(self.banlist_path))
        self.connect_only = connect_only
        self.max_outbound = max_outbound
        self.proxies = ProxyTable()          # -proxy / -onion / -onlynet (netbase SetProxy / SetLimited)
        self.whitelist: list = []            # -whitelist subnets (ipaddress networks)
        self.blocks_only = False             # -blocksonly: no transaction relay in either direction
        self.peer_bloom_filters = True       # -peerbloomfilters: NODE_BLOOM and the BIP37 messages
        self.whitelist_relay = True          # -whitelistrelay: whitelisted peers' txs even with -blocksonly
        self.whitelist_force_relay = True    # -whitelistforcerelay: re-announce their txs we already have
        self.user_agent = P.USER_AGENT       # with -uacomment
        # orphan transactions (mapOrphanTransactions): txid -> (tx, peer id, expiry), -maxorphantx
        self.orphans: dict[bytes, tuple] = {}
        self.orphans_by_prev: dict[tuple[bytes, int], set[bytes]] = {}
        self.max_orphans = DEFAULT_MAX_ORPHAN_TRANSACTIONS
        self.timedata = TimeData()           # -maxtimeadjustment
        self.max_outbound_limit = 0          # -maxuploadtarget (bytes per 24 h cycle; 0 = none)
        self.max_outbound_timeframe = 24 * 60 * 60
        self.outbound_cycle_start = 0.0
        self.outbound_cycle_bytes = 0
        self.dns_seeds: list[str] = []       # chainparams vSeeds (-dnsseed / -forcednsseed)
        self.force_dns_seed = False
        self._orphan_lock = threading.RLock()
        self.local_addrs: dict[tuple[str, int], int] = {}  # AddLocal: (host, port) -> score

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
        for host, port, white in self.extra_binds:
            srv = socket.socket(socket.AF_INET6 if ":" in host else socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((host, port))
            srv.listen(16)
            self._extra_servers.append(srv)
            threading.Thread(target=self._accept_loop, args=(srv, white), name="p2p-listen", daemon=True).start()
            log.log_printf(f"P2P listening on {host}:{srv.getsockname()[1]}{' (whitelisted)' if white else ''}")
        if not self.connect_only and self.max_outbound > 0:
            threading.Thread(target=self._open_connections, name="p2p-opencon", daemon=True).start()
        if self.dns_seeds and not self.connect_only:
            threading.Thread(target=self.dns_address_seed, name="p2p-dnsseed", daemon=True).start()

    def dns_address_seed(self, resolve=None) -> int:
        """ThreadDNSAddressSeed: unless the address manager already knows peers (and -forcednsseed
        is off), resolve every DNS seed to addresses on the default port and add them to addrman
        with the seed as their source. Returns the number of addresses added."""
        if self.addrman.size() > 0 and not self.force_dns_seed:
            log.log_print("net", "P2P peers available. Skipped DNS seeding.")
            return 0
        resolve = resolve or socket.getaddrinfo
        found = 0
        for seed in self.dns_seeds:
            try:
                infos = resolve(seed, self.params.default_port, socket.AF_INET, socket.SOCK_STREAM)
            except OSError as e:
                log.log_print("net", f"DNS seed {seed} unavailable: {e}")
                continue
            now = int(time.time())
            # seed addresses are stamped 3-7 days old, as the reference does, so they rank low
            entries = [(info[4][0], self.params.default_port, P.NODE_NETWORK, now - 3 * 86400 - random.randrange(4 * 86400))
                       for info in infos]
            found += self.addrman.add(entries, seed) or 0
        log.log_printf(f"{found} addresses found from DNS seeds")
        return found

    def _open_connections(self) -> None:
        """ThreadOpenConnections: keep up to max_outbound outbound peers, picked from addrman."""
        while not self._stop.wait(0.5):
            if not self.network_active:
                continue
            with self._lock:
                outbound = sum(1 for p in self.peers if not p.inbound)
                connected = {f"{p.addr[0]}:{p.addr[1]}" for p in self.peers}
            if outbound >= self.max_outbound or self.addrman.size() == 0:
                continue
            pick = self.addrman.select(exclude=connected)
            if pick is None or self.is_banned(pick[0]) or (self.port and pick == ("127.0.0.1", self.port)):
                continue
            self.addrman.attempt(*pick)
            try:
                self.connect(pick[0], pick[1], timeout=3.0)
            except OSError:
                continue

    def _accept_loop(self, srv: socket.socket | None = None, white: bool = False) -> None:
        srv = srv or self._server
        while not self._stop.is_set():
            try:
                sock, addr = srv.accept()
            except OSError:
                break
            if not self.network_active or (self.is_banned(addr[0]) and not white):
                sock.close()  # CConnman::AcceptConnection drops banned / inactive-network peers
                continue
            self._add(sock, addr, inbound=True, whitebind=white)

    def connect(self, host: str, port: int, timeout: float = 10.0) -> Peer:
        if not self.network_active:
            raise ConnectionError("network is disabled (setnetworkactive false)")
        if not self.allow_dns and not host.endswith(".onion"):
            try:
                ipaddress.ip_address(host)
            except ValueError:  # -dns=0: names are not looked up (Lookup's fAllowLookup)
                raise ConnectionError(f"cannot connect to {host}: DNS lookups are disabled (-dns=0)") from None
        sock = self.proxies.connect(host, port, timeout=timeout)  # direct, or SOCKS5 through the net's proxy
        sock.settimeout(None)
        return self._add(sock, (host, port), inbound=False)

    @property
    def local_services(self) -> int:
        # a pruning node cannot serve the whole chain: no NODE_NETWORK (src/init.cpp, fPruneMode)
        network = 0 if getattr(self.state, "prune_mode", False) else P.NODE_NETWORK
        return network | P.NODE_WITNESS | (P.NODE_BLOOM if self.peer_bloom_filters else 0)

    def is_whitelisted(self, ip: str) -> bool:
        try:
            a = ipaddress.ip_address(ip)
        except ValueError:
            return False
        return any(a.version == n.version and a in n for n in self.whitelist)

    def discover_local_addresses(self, resolve=None) -> int:
        """Discover(): the host's own addresses (by hostname lookup) that are routable, added with
        LOCAL_IF score; loopback, private and link-local addresses are skipped (IsRoutable)."""
        resolve = resolve or (lambda: socket.getaddrinfo(socket.gethostname(), None))
        try:
            infos = resolve()
        except OSError:
            return 0
        n = 0
        for info in infos:
            ip = info[4][0]
            try:
                a = ipaddress.ip_address(ip.split("%")[0])
            except ValueError:
                continue
            if a.is_global:
                self.add_local(str(a), self.port or self.params.default_port, 1)
                n += 1
        return n

    # ---------------------------------------------------------------- -maxuploadtarget
    def record_sent(self, n: int) -> None:
        """RecordBytesSent: bytes in the current upload cycle (a new cycle every timeframe)."""
        now = time.time()
        if now > self.outbound_cycle_start + self.max_outbound_timeframe:
            self.outbound_cycle_start, self.outbound_cycle_bytes = now, 0
        self.outbound_cycle_bytes += n

    def outbound_target_reached(self, historical_only: bool) -> bool:
        """OutboundTargetReached: with `historical_only`, true once less than one MAX_BLOCK_SERIALIZED
        buffer of the target is left (recent blocks are still served until the target itself)."""
        if not self.max_outbound_limit:
            return False
        if historical_only:
            buffer = self.max_outbound_timeframe // 600 * 8_000_000  # MAX_BLOCK_SERIALIZED_SIZE per expected block
            return buffer >= self.max_outbound_limit or self.outbound_cycle_bytes >= self.max_outbound_limit - buffer
        return self.outbound_cycle_bytes >= self.max_outbound_limit

    def upload_target_info(self) -> dict:
        now = time.time()
        left_t = max(0, int(self.outbound_cycle_start + self.max_outbound_timeframe - now)) if self.max_outbound_limit else 0
        return {"timeframe": self.max_outbound_timeframe, "target": self.max_outbound_limit,
                "target_reached": self.outbound_target_reached(False),
                "serve_historical_blocks": not self.outbound_target_reached(True),
                "bytes_left_in_cycle": max(0, self.max_outbound_limit - self.outbound_cycle_bytes)
                if self.max_outbound_limit else 0,
                "time_left_in_cycle": left_t}

    def add_local(self, host: str, port: int, score: int = 1) -> None:
        """AddLocal (src/net.cpp): an address this node is reachable at, e.g. its onion service."""
        with self._lock:
            self.local_addrs[(host, port)] = max(score, self.local_addrs.get((host, port), 0))

    def remove_local(self, host: str, port: int) -> None:
        with self._lock:
            self.local_addrs.pop((host, port), None)

    def _add(self, sock, addr, inbound: bool, whitebind: bool = False) -> Peer:
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, max(4096, self.max_receive_buffer))
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, max(4096, self.max_send_buffer))
        p = Peer(self, sock, addr, inbound)
        p.whitebind = whitebind
        with self._lock:
            self.peers.append(p)
        p.thread.start()
        return p

    def remove(self, p: Peer) -> None:
        with self._lock:
            if p in self.peers:
                self.peers.remove(p)
        self.erase_orphans_for(p.id)  # FinalizeNode -> EraseOrphansFor

    # ---------------------------------------------------------------- orphan transactions
    def add_orphan(self, tx, peer_id: int) -> bool:
        """AddOrphanTx: keep a transaction whose inputs are unknown (at most MAX_STANDARD_TX_WEIGHT,
        expiring after ORPHAN_TX_EXPIRE_TIME), then LimitOrphanTxSize to -maxorphantx."""
        txid = tx.txid()
        with self._orphan_lock:
            if txid in self.orphans:
                return False
            if len(tx.serialize(False)) * 3 + len(tx.serialize(True)) > MAX_ORPHAN_TX_WEIGHT:
                log.log_print("mempool", f"ignoring large orphan tx {_core.u256_hex(txid)}")
                return False
            self.orphans[txid] = (tx, peer_id, time.time() + ORPHAN_TX_EXPIRE_TIME)
            for i in tx.vin:
                self.orphans_by_prev.setdefault((i.prevout.hash, i.prevout.n), set()).add(txid)
            self.limit_orphans()
        return True

    def erase_orphan(self, txid: bytes) -> None:
        with self._orphan_lock:
            ent = self.orphans.pop(txid, None)
            if ent is None:
                return
            for i in ent[0].vin:
                s = self.orphans_by_prev.get((i.prevout.hash, i.prevout.n))
                if s is not None:
                    s.discard(txid)
                    if not s:
                        del self.orphans_by_prev[(i.prevout.hash, i.prevout.n)]

    def erase_orphans_for(self, peer_id: int) -> None:
        with self._orphan_lock:
            for t in [t for t, e in self.orphans.items() if e[1] == peer_id]:
                self.erase_orphan(t)

    def limit_orphans(self) -> int:
        """LimitOrphanTxSize: drop expired orphans, then random ones above the limit."""
        now, gone = time.time(), 0
        with self._orphan_lock:
            for t in [t for t, e in self.orphans.items() if e[2] <= now]:
                self.erase_orphan(t)
                gone += 1
            while len(self.orphans) > self.max_orphans:
                self.erase_orphan(random.choice(list(self.orphans)))
                gone += 1
        return gone

    def process_orphans(self, parent_txid: bytes, n_out: int) -> list[bytes]:
        """The ProcessMessage("tx") work queue: orphans spending a newly accepted transaction are
        retried; accepted ones queue their own children, invalid ones are dropped."""
        accepted, work = [], [(parent_txid, n_out)]
        while work:
            txid, n = work.pop()
            for k in range(n):
                with self._orphan_lock:
                    kids = list(self.orphans_by_prev.get((txid, k), ()))
                for o in kids:
                    with self._orphan_lock:
                        ent = self.orphans.get(o)
                    if ent is None:
                        continue
                    ok, reason, _ = self.state.accept_to_mempool(ent[0])
                    if ok:
                        accepted.append(o)
                        self.erase_orphan(o)
                        work.append((o, len(ent[0].vout)))
                    elif reason != "missing-inputs":
                        self.erase_orphan(o)
        return accepted

    def stop(self) -> None:
        self._stop.set()
        try:
            self.addrman.save()
            if self.banlist_path:
                save_banlist(self.banlist_path, self.banned)
        except OSError as e:
            log.log_printf(f"could not write peers.dat / banlist.dat: {e}")
        if self._server is not None:
            self._server.close()
        for srv in self._extra_servers:
            srv.close()
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
        if self.banlist_path:
            save_banlist(self.banlist_path, self.banned)
        for p in list(self.peers):
            if p.addr[0] == address:
                p.close()

    def unban(self, address: str) -> bool:
        gone = self.banned.pop(address, None) is not None
        if gone and self.banlist_path:
            save_banlist(self.banlist_path, self.banned)
        return gone

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
    def announce_block(self, header, block=None) -> None:
        """New tip: `cmpctblock` to high-bandwidth BIP152 peers, `headers` to peers that asked for
        sendheaders, `inv` to the rest."""
        act = self.params.kawpow_activation_time
        h = self.state.block_hash(header)
        cmpct = None
        for p in list(self.peers):
            if not p.verack:
                continue
            try:
                if p.cmpct_hb and block is not None:
                    if cmpct is None:
                        cmpct = CompactBlock.from_block(block, act).payload()
                    p.send("cmpctblock", cmpct)
                elif p.send_headers:
                    p.send("headers", _core.headers_msg_encode([header], act))
                else:
                    p.send("inv", P.inv_payload([(P.MSG_BLOCK, h)]))
            except OSError:
                p.close()

    def announce_tx(self, txid: bytes, skip: "Peer | None" = None) -> None:
        """RelayTransaction: `inv` MSG_TX to every peer that has not sent us this tx."""
        tx = None
        for p in list(self.peers):
            if p is skip or not p.verack or not p.relay_txs or txid in p.known_txs:
                continue
            if p.bloom is not None:  # BIP37: relay only what the peer's filter matches
                if tx is None:
                    e = self.state.mempool.get(txid)
                    tx = e.tx if e is not None else None
                if tx is None or not p.bloom.is_relevant_and_update(tx):
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
        # AddTimeData: outbound peers' clocks feed the network-adjusted time
        offset = int(info.get("time", 0)) - int(time.time())
        peer.info["timeoffset"] = offset
        if not peer.inbound:
            self.state.time_offset = self.timedata.add(peer.addr[0], offset)
        if peer.inbound and not peer.sent_version:
            peer.send_version()
        peer.send("verack")
        if not peer.inbound:  # an outbound peer that answered is a good address (MarkAddressGood)
            self.addrman.good(peer.addr[0], peer.addr[1])

    def on_verack(self, peer: Peer, p: bytes) -> None:
        peer.verack = True
        peer.send("sendheaders")
        peer.send("sendcmpct", struct.pack("<?Q", False, 2))  # BIP152 v2, low-bandwidth
        if not peer.inbound:
            peer.send("getaddr")
        self.request_headers(peer)

    # ---------------------------------------------------------------- addresses (N4)
    def on_addr(self, peer: Peer, p: bytes) -> None:
        entries = _parse_addr(p)
        if len(entries) > MAX_ADDR_TO_SEND:
            peer.misbehaving(20, "oversized addr")
            return
        now = int(time.time())
        fresh = [(ip, port, s, t if 100000000 < t <= now + 600 else now - 5 * 86400) for ip, port, s, t in entries]
        self.addrman.add(fresh, peer.addr[0], penalty=2 * 3600)
        if len(entries) <= 10:  # RelayAddress: small, fresh announcements go on to two peers
            relay = [e for e in fresh if e[3] > now - 600]
            others = [q for q in self.peers if q is not peer and q.verack]
            for q in random.sample(others, min(2, len(others))) if relay else []:
                try:
                    q.send("addr", _ser_addr(relay))
                except OSError:
                    q.close()

    def on_getaddr(self, peer: Peer, p: bytes) -> None:
        """Answered once, for inbound peers only (fingerprinting protection, net_processing.cpp)."""
        if not peer.inbound or peer.getaddr_answered:
            return
        peer.getaddr_answered = True
        items = [(a.ip, a.port, a.services, a.time) for a in self.addrman.get_addr()]
        for k in range(0, len(items), MAX_ADDR_TO_SEND):
            peer.send("addr", _ser_addr(items[k:k + MAX_ADDR_TO_SEND]))

    # ---------------------------------------------------------------- BIP37 (N5)
    def _bloom_allowed(self, peer: Peer) -> bool:
        """-peerbloomfilters=0: BIP111 says a peer asking for a filter we do not serve goes."""
        if self.peer_bloom_filters:
            return True
        peer.misbehaving(100, "bloom filter message while NODE_BLOOM is off")
        return False

    def on_filterload(self, peer: Peer, p: bytes) -> None:
        if not self._bloom_allowed(peer):
            return
        f = BloomFilter.from_payload(p)
        if not f.within_size_constraints():
            peer.misbehaving(100, "oversized bloom filter")
            return
        peer.bloom = f
        peer.info["relay"] = True

    def on_filteradd(self, peer: Peer, p: bytes) -> None:
        n, off = P.de_compact(p, 0)
        data = p[off:off + n]
        if len(data) > MAX_SCRIPT_ELEMENT_SIZE or peer.bloom is None:
            peer.misbehaving(100, "bad filteradd")
            return
        peer.bloom.insert(data)

    def on_filterclear(self, peer: Peer, p: bytes) -> None:
        peer.bloom = None
        peer.info["relay"] = True

    # ---------------------------------------------------------------- BIP152 (N5)
    def on_sendcmpct(self, peer: Peer, p: bytes) -> None:
        announce, version = struct.unpack_from("<?Q", p, 0)
        if version in (1, 2) and version >= peer.cmpct_version:
            peer.cmpct_version = version
            peer.cmpct_hb = bool(announce)

    def on_cmpctblock(self, peer: Peer, p: bytes) -> None:
        act = self.params.kawpow_activation_time
        cb = CompactBlock.from_payload(p, act)
        h = self.state.block_hash(cb.header)
        if h in self.state.block_pos:
            return
        if self.state.chain.find(cb.header.prev) is None:
            self.request_headers(peer)
            return
        with self.state.lock:
            pool = [e.tx for e in self.state.mempool.values()]
        pool += list(self.extra_txn)  # PartiallyDownloadedBlock::InitData's extra_txn
        slots, missing = cb.reconstruct(pool, peer.cmpct_version or 2)
        if missing:
            peer.partial[h] = (cb, slots)
            peer.send("getblocktxn", getblocktxn_payload(h, missing))
            REGISTRY.inc("p2p_cmpct_getblocktxn_total", 1)
            return
        self._finish_compact(peer, cb, slots)

    def _finish_compact(self, peer: Peer, cb, slots) -> None:
        blk = _core.Block()
        blk.header = cb.header
        blk.vtx = slots
        root, _ = blk.merkle_root()
        if root != cb.header.merkle_root:  # a short-id collision built the wrong block: fetch it whole
            peer.send("getdata", P.inv_payload([(P.MSG_BLOCK | P.MSG_WITNESS_FLAG, self.state.block_hash(cb.header))]))
            return
        REGISTRY.inc("p2p_cmpct_reconstructed_total", 1)
        self.state.arm_reorg_guard(self.peer_count())
        st = self.state.process_new_block(blk)
        if not st.ok and st.reject != "duplicate":
            peer.misbehaving(st.dos or 0, f"invalid compact block: {st.reject}")

    def on_getblocktxn(self, peer: Peer, p: bytes) -> None:
        h, idx = parse_getblocktxn(p)
        blk = self.state.get_block(h)
        if blk is None:
            return
        vtx = list(blk.vtx)
        if any(i >= len(vtx) for i in idx):
            peer.misbehaving(100, "getblocktxn with out-of-bounds tx indices")
            return
        peer.send("blocktxn", blocktxn_payload(h, [vtx[i] for i in idx]))

    def on_blocktxn(self, peer: Peer, p: bytes) -> None:
        h, txs = parse_blocktxn(p)
        pending = peer.partial.pop(h, None)
        if pending is None:
            return
        cb, slots = pending
        missing = [i for i, t in enumerate(slots) if t is None]
        if len(txs) != len(missing):
            peer.misbehaving(100, "blocktxn does not fill the block")
            return
        for i, t in zip(missing, txs):
            slots[i] = t
        self._finish_compact(peer, cb, slots)

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
        from ..models.verify import process_batch_resident, process_headers, resident_ready

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
            res = None
            act = self.params.kawpow_activation_time
            if self.gpus and resident_ready(headers, act, self.gpus[0], self.verify_mode):
                # one upload, PoW + block hashes + DGW nBits on the GPU, one download, the bulk
                # insert on the host (None: not height-ordered -> the staged path below)
                res = process_batch_resident(chain, _core.HeaderBatch.from_headers(headers, act),
                                             self.state.adjusted_time(), device=self.gpus[0])
                if res is not None:
                    REGISTRY.inc("p2p_headers_resident_total", len(headers))
            if res is None:
                res = process_headers(chain, headers, self.state.adjusted_time(), gpus=self.gpus,
                                      mode=self.verify_mode)
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
        if self.blocks_only and not (peer.whitelisted and self.whitelist_relay):  # fBlocksOnly
            log.log_print("net", f"transaction sent in violation of protocol peer={peer.id}")
            return
        tx = _core.Transaction.deserialize(p)
        txid = tx.txid()
        peer.known_txs.add(txid)
        REGISTRY.inc("p2p_tx_received_total", 1)
        if txid in self.state.mempool:
            if peer.whitelisted and self.whitelist_force_relay:  # -whitelistforcerelay
                self.announce_tx(txid)
            return
        self.state.last_replaced = []
        ok, reason, _ = self.state.accept_to_mempool(tx)
        if ok:
            if self.extra_txn.maxlen:  # transactions a replacement pushed out stay usable for compact blocks
                self.extra_txn.extend(self.state.last_replaced)
            self.process_orphans(txid, len(tx.vout))
            return
        if reason == "missing-inputs":
            if self.extra_txn.maxlen:
                self.extra_txn.append(tx)
            # keep it as an orphan and ask the sender for the parents we do not have
            missing = [i.prevout.hash for i in tx.vin
                       if i.prevout.hash not in self.state.mempool and i.prevout.hash not in self.orphans]
            if self.add_orphan(tx, peer.id) and missing:
                peer.send("getdata", P.inv_payload([(P.MSG_TX, h) for h in dict.fromkeys(missing)]))
            return
        REGISTRY.inc("p2p_tx_rejected_total", 1)
        log.log_print("mempool", f"tx {_core.u256_hex(txid)} from peer {peer.id} rejected: {reason}")
        if self.extra_txn.maxlen:  # a policy reject may still be in a block
            self.extra_txn.append(tx)

    def on_mempool(self, peer: Peer, p: bytes) -> None:
        """BIP35: inv of every pool txid (in MAX_INV_SZ chunks), through the peer's bloom filter."""
        ids = [h for h, e in list(self.state.mempool.items())
               if peer.bloom is None or peer.bloom.is_relevant_and_update(e.tx)]
        peer.known_txs.update(ids)
        for k in range(0, len(ids), P.MAX_INV_SZ):
            peer.send("inv", P.inv_payload([(P.MSG_TX, h) for h in ids[k:k + P.MAX_INV_SZ]]))

    def on_feefilter(self, peer: Peer, p: bytes) -> None:
        (peer.fee_filter,) = struct.unpack_from("<q", p, 0)

    def on_getdata(self, peer: Peer, p: bytes) -> None:
        missing = []
        act = self.params.kawpow_activation_time
        for t, h in P.parse_inv(p):
            kind = t & ~P.MSG_WITNESS_FLAG
            if kind == MSG_FILTERED_BLOCK or kind == MSG_CMPCT_BLOCK:
                blk = self.state.get_block(h)
                if blk is None:
                    missing.append((t, h))
                elif kind == MSG_CMPCT_BLOCK:
                    peer.send("cmpctblock", CompactBlock.from_block(blk, act, peer.cmpct_version or 2).payload())
                elif peer.bloom is not None:  # merkleblock, then the matched transactions
                    payload, matched = merkle_block(blk, blk.header.serialize(act), peer.bloom)
                    peer.send("merkleblock", payload)
                    for tx in matched:
                        if tx.txid() not in peer.known_txs:
                            peer.send("tx", tx.serialize(False))
                continue
            if kind == P.MSG_BLOCK:
                idx = self.state.chain.find(h)
                historical = idx is not None and idx.time < time.time() - 7 * 24 * 3600
                if historical and not peer.whitelisted and self.outbound_target_reached(True):
                    # historical block serving limit reached: disconnect (ProcessGetData)
                    log.log_print("net", f"historical block serving limit reached, disconnect peer={peer.id}")
                    peer.close()
                    return
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
