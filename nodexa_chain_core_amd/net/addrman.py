"""Peer address manager: CAddrMan's new / tried tables, peers.dat and banlist.dat.

Parity (behaviour): CAddrMan (src/addrman.h:185, src/addrman.cpp) — addresses learnt from `addr`
messages go to a "new" table bucketed by (source group, address group) under a secret key,
addresses we connected to successfully move to a "tried" table bucketed by address group, Select()
picks tried or new with equal odds (biased towards fresh, rarely-failed entries), GetAddr() returns
a random 23 % (at most 2500) of the known addresses, terrible entries (too old, too many failures)
are skipped. Buckets are chosen with SipHash keyed by the per-node secret, as the reference does
with its nKey, so an attacker cannot target one bucket. peers.dat / banlist.dat here are JSON with
a SHA256d checksum (CAddrDB / CBanDB write the serialized tables with the same kind of checksum).
"""
from __future__ import annotations

import hashlib
import ipaddress
import json
import os
import random
import threading
import time

from .. import core

_core = core()

NEW_BUCKETS, TRIED_BUCKETS, BUCKET_SIZE = 1024, 256, 64
NEW_BUCKETS_PER_SOURCE_GROUP = 64
TRIED_BUCKETS_PER_GROUP = 8
HORIZON_DAYS = 30             # ADDRMAN_HORIZON_DAYS
RETRIES = 3                   # ADDRMAN_RETRIES
MAX_FAILURES = 10             # ADDRMAN_MAX_FAILURES
MIN_FAIL_DAYS = 7             # ADDRMAN_MIN_FAIL_DAYS
GETADDR_MAX_PCT, GETADDR_MAX = 23, 2500


def group(ip: str) -> bytes:
    """GetGroup: /16 for IPv4, /32 for IPv6, the whole address for local ones."""
    try:
        a = ipaddress.ip_address(ip)
    except ValueError:
        return ip.encode()
    if a.is_loopback or a.is_private:
        return b"\x00" + a.packed
    if a.version == 4:
        return b"\x01" + a.packed[:2]
    return b"\x02" + a.packed[:4]


class AddrInfo:
    __slots__ = ("ip", "port", "services", "time", "source", "last_try", "last_success", "attempts", "tried")

    def __init__(self, ip: str, port: int, services: int, t: int, source: str):
        self.ip, self.port, self.services, self.time, self.source = ip, port, services, t, source
        self.last_try = self.last_success = 0
        self.attempts = 0
        self.tried = False

    @property
    def key(self) -> str:
        return f"{self.ip}:{self.port}"

    def is_terrible(self, now: int) -> bool:
        """IsTerrible: tried in the last minute never counts; too old, future, or failing."""
        if self.last_try and self.last_try >= now - 60:
            return False
        if self.time > now + 10 * 60 or self.time == 0 or now - self.time > HORIZON_DAYS * 86400:
            return True
        if self.last_success == 0 and self.attempts >= RETRIES:
            return True
        return now - self.last_success > MIN_FAIL_DAYS * 86400 and self.attempts >= MAX_FAILURES

    def chance(self, now: int) -> float:
        """GetChance: lower for recently tried and failing entries."""
        c = 1.0
        if now - self.last_try < 10 * 60:
            c *= 0.01
        return c * 0.66 ** min(self.attempts, 8)


class AddrMan:
    def __init__(self, path: str | None = None, key: bytes | None = None):
        self.path = path
        self.key = key or os.urandom(32)
        self.lock = threading.RLock()
        self.info: dict[str, AddrInfo] = {}
        self.new: dict[int, dict[int, str]] = {}    # bucket -> position -> address key
        self.tried: dict[int, dict[int, str]] = {}
        if path and os.path.exists(path):
            self.load()

    # ------------------------------------------------------------------ bucketing
    def _hash(self, *parts: bytes) -> int:
        k0 = int.from_bytes(self.key[:8], "little")
        k1 = int.from_bytes(self.key[8:16], "little")
        return _core.siphash24(k0, k1, b"".join(parts))

    def _new_bucket(self, a: AddrInfo) -> int:
        h1 = self._hash(group(a.ip), group(a.source)) % NEW_BUCKETS_PER_SOURCE_GROUP
        return self._hash(group(a.source), h1.to_bytes(8, "little")) % NEW_BUCKETS

    def _tried_bucket(self, a: AddrInfo) -> int:
        h1 = self._hash(a.key.encode()) % TRIED_BUCKETS_PER_GROUP
        return self._hash(group(a.ip), h1.to_bytes(8, "little")) % TRIED_BUCKETS

    def _position(self, a: AddrInfo, new: bool, bucket: int) -> int:
        return self._hash(b"N" if new else b"K", bucket.to_bytes(4, "little"), a.key.encode()) % BUCKET_SIZE

    def _place(self, table: dict, bucket: int, pos: int, key: str) -> None:
        old = table.setdefault(bucket, {}).get(pos)
        if old is not None and old != key:
            o = self.info.get(old)
            if o is not None and not o.is_terrible(int(time.time())) and table is self.new:
                return  # keep a good occupant (the reference only replaces terrible ones)
            self._forget(old)
        table[bucket][pos] = key

    def _forget(self, key: str) -> None:
        self.info.pop(key, None)
        for table in (self.new, self.tried):
            for b in table.values():
                for p in [p for p, k in b.items() if k == key]:
                    del b[p]

    # ------------------------------------------------------------------ API
    def size(self) -> int:
        with self.lock:
            return len(self.info)

    def add(self, addrs: list[tuple[str, int, int, int]], source: str, penalty: int = 0) -> int:
        """Add(): (ip, port, services, time) entries heard from `source`; returns how many were new."""
        n = 0
        now = int(time.time())
        with self.lock:
            for ip, port, services, t in addrs:
                try:
                    ipaddress.ip_address(ip)
                except ValueError:
                    continue
                if port == 0:
                    continue
                key = f"{ip}:{port}"
                a = self.info.get(key)
                t = max(0, min(int(t), now + 600) - penalty)
                if a is not None:
                    a.services |= services
                    a.time = max(a.time, t)
                    continue
                a = AddrInfo(ip, port, services, t, source)
                self.info[key] = a
                b = self._new_bucket(a)
                self._place(self.new, b, self._position(a, True, b), key)
                if key in self.info:
                    n += 1
        return n

    def good(self, ip: str, port: int) -> None:
        """Good(): a successful connection moves the entry to the tried table."""
        key = f"{ip}:{port}"
        now = int(time.time())
        with self.lock:
            a = self.info.get(key)
            if a is None:
                self.add([(ip, port, 0, now)], ip)
                a = self.info.get(key)
                if a is None:
                    return
            a.last_success = a.time = now
            a.last_try = now
            a.attempts = 0
            if a.tried:
                return
            for b in self.new.values():
                for p in [p for p, k in b.items() if k == key]:
                    del b[p]
            a.tried = True
            tb = self._tried_bucket(a)
            pos = self._position(a, False, tb)
            evicted = self.tried.setdefault(tb, {}).get(pos)
            if evicted is not None and evicted != key and evicted in self.info:  # back to the new table
                e = self.info[evicted]
                e.tried = False
                nb = self._new_bucket(e)
                self._place(self.new, nb, self._position(e, True, nb), evicted)
            self.tried[tb][pos] = key

    def attempt(self, ip: str, port: int) -> None:
        with self.lock:
            a = self.info.get(f"{ip}:{port}")
            if a is not None:
                a.last_try = int(time.time())
                a.attempts += 1

    def select(self, new_only: bool = False, exclude: set | None = None) -> tuple[str, int] | None:
        """Select(): tried or new with even odds, then an entry weighted by its chance."""
        now = int(time.time())
        with self.lock:
            pools = []
            tried = [k for b in self.tried.values() for k in b.values()]
            new = [k for b in self.new.values() for k in b.values()]
            if not new_only and tried:
                pools.append(tried)
            if new:
                pools.append(new)
            if not pools:
                return None
            random.shuffle(pools)
            for pool in pools:
                cands = [self.info[k] for k in pool if k in self.info and (not exclude or k not in exclude)]
                if not cands:
                    continue
                for _ in range(64):
                    a = random.choice(cands)
                    if random.random() < a.chance(now):
                        return a.ip, a.port
                return cands[0].ip, cands[0].port
            return None

    def get_addr(self) -> list[AddrInfo]:
        """GetAddr(): a random 23 % (max 2500) of the non-terrible entries."""
        now = int(time.time())
        with self.lock:
            good = [a for a in self.info.values() if not a.is_terrible(now)]
        random.shuffle(good)
        n = min(GETADDR_MAX, len(self.info) * GETADDR_MAX_PCT // 100) or min(len(good), 1)
        return good[:n]

    # ------------------------------------------------------------------ peers.dat
    def save(self) -> None:
        if not self.path:
            return
        with self.lock:
            body = json.dumps({"key": self.key.hex(), "addrs": [
                {"ip": a.ip, "port": a.port, "services": a.services, "time": a.time, "source": a.source,
                 "last_try": a.last_try, "last_success": a.last_success, "attempts": a.attempts, "tried": a.tried}
                for a in self.info.values()]}).encode()
        _write_checked(self.path, body)

    def load(self) -> bool:
        body = _read_checked(self.path)
        if body is None:
            return False
        d = json.loads(body)
        self.key = bytes.fromhex(d["key"])
        for e in d["addrs"]:
            a = AddrInfo(e["ip"], e["port"], e["services"], e["time"], e["source"])
            a.last_try, a.last_success, a.attempts = e["last_try"], e["last_success"], e["attempts"]
            self.info[a.key] = a
            if e["tried"]:
                a.tried = True
                tb = self._tried_bucket(a)
                self.tried.setdefault(tb, {})[self._position(a, False, tb)] = a.key
            else:
                nb = self._new_bucket(a)
                self.new.setdefault(nb, {})[self._position(a, True, nb)] = a.key
        return True


def _write_checked(path: str, body: bytes) -> None:
    """File = body || sha256d(body), written atomically (CAddrDB::Write / CBanDB::Write)."""
    tmp = path + ".new"
    with open(tmp, "wb") as f:
        f.write(body + hashlib.sha256(hashlib.sha256(body).digest()).digest())
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def _read_checked(path: str) -> bytes | None:
    try:
        with open(path, "rb") as f:
            raw = f.read()
    except OSError:
        return None
    body, check = raw[:-32], raw[-32:]
    if len(raw) < 32 or hashlib.sha256(hashlib.sha256(body).digest()).digest() != check:
        return None
    return body


def save_banlist(path: str, banned: dict) -> None:
    _write_checked(path, json.dumps(banned).encode())


def load_banlist(path: str) -> dict:
    body = _read_checked(path)
    return json.loads(body) if body is not None else {}
