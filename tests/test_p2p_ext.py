"""Address manager (N4), BIP37 bloom filters / merkleblock and BIP152 compact blocks (N5): unit
checks (the reference's bloom_tests.cpp filter vectors used as data) and two-node / raw-socket
exchanges over localhost."""
import socket
import struct
import time

import pytest

from nodexa_chain_core_amd.net import protocol as P
from nodexa_chain_core_amd.net.addrman import AddrMan
from nodexa_chain_core_amd.net.bloom import BLOOM_UPDATE_ALL, BloomFilter
from nodexa_chain_core_amd.net.compact import CompactBlock, parse_getblocktxn, getblocktxn_payload
from nodexa_chain_core_amd.net.p2p import _parse_addr, _ser_addr
from nodexa_chain_core_amd.utils.metrics import REGISTRY
from test_p2p import _node, _wait


def test_bloom_filter_reference_vectors():
    for tweak, expect in ((0, "03614e9b050000000000000001"), (2147483649, "03ce4299050000000100008001")):
        f = BloomFilter.create(3, 0.01, tweak, BLOOM_UPDATE_ALL)
        f.insert(bytes.fromhex("99108ad8ed9bb6274d3980bab5a85c048f0950c8"))
        assert f.contains(bytes.fromhex("99108ad8ed9bb6274d3980bab5a85c048f0950c8"))
        assert not f.contains(bytes.fromhex("19108ad8ed9bb6274d3980bab5a85c048f0950c8"))
        f.insert(bytes.fromhex("b5a2c786d9ef4658287ced5914b37a1b4aa32eee"))
        f.insert(bytes.fromhex("b9300670b4c5366e95b2699e8b18bc75e5f729c5"))
        assert f.payload().hex() == expect
        assert BloomFilter.from_payload(f.payload()).payload() == f.payload()


def test_addrman_tables_and_persistence(tmp_path):
    am = AddrMan(str(tmp_path / "peers.dat"))
    now = int(time.time())
    n = am.add([(f"10.{i // 250}.{i % 250}.1", 8788, 1, now - 60) for i in range(300)] +
               [("203.0.113.9", 8788, 1, now - 60)], "198.51.100.1")
    assert n >= 250 and am.size() == n  # a few collide in their new bucket and are dropped
    assert am.add([("not-an-ip", 1, 1, now)], "x") == 0
    am.good("203.0.113.9", 8788)
    assert am.info["203.0.113.9:8788"].tried
    assert am.select() is not None
    sample = am.get_addr()
    assert 0 < len(sample) <= max(1, am.size() * 23 // 100)
    am.attempt("203.0.113.9", 8788)
    am.save()
    am2 = AddrMan(str(tmp_path / "peers.dat"))
    assert am2.size() == am.size() and am2.info["203.0.113.9:8788"].tried and am2.key == am.key
    # addr wire format round trip (IPv4-mapped IPv6, big-endian port)
    raw = _ser_addr([("203.0.113.9", 8788, 9, now)])
    assert _parse_addr(raw) == [("203.0.113.9", 8788, 9, now)]


def test_compact_block_encoding_and_reconstruction(core):
    from nodexa_chain_core_amd.utils.synth_block import make_signed_block

    blk, _, _ = make_signed_block(12, seed=5, witness_every=3)
    hdr = core.BlockHeader()
    hdr.version, hdr.time, hdr.bits = 0x30000000, 1600000000, 0x207FFFFF
    root, _ = blk.merkle_root()
    hdr.merkle_root = root
    blk.header = hdr
    act = 2**31
    cb = CompactBlock.from_block(blk, act, nonce=7)
    back = CompactBlock.from_payload(cb.payload(), act)
    assert back.shortids == cb.shortids and back.nonce == 7 and len(back.prefilled) == 1
    txs = list(blk.vtx)
    slots, missing = back.reconstruct(txs[1:])
    assert missing == [] and [t.txid() for t in slots] == [t.txid() for t in txs]
    slots, missing = back.reconstruct(txs[1:4] + txs[6:])
    assert missing == [4, 5]
    h, idx = parse_getblocktxn(getblocktxn_payload(b"\x01" * 32, [4, 5, 9]))
    assert h == b"\x01" * 32 and idx == [4, 5, 9]


def test_compact_block_rejects_oversized_counts(core):
    """A ~90-byte cmpctblock declaring 2^64-1 short ids must be refused before any allocation
    (the reference's deserialiser fails at end of stream); same for getblocktxn / blocktxn."""

    from nodexa_chain_core_amd.net.bloom import _ser_compact
    from nodexa_chain_core_amd.net.compact import parse_blocktxn

    hdr = core.BlockHeader()
    hdr.version, hdr.time, hdr.bits = 0x30000000, 1600000000, 0x207FFFFF
    act = 2**31
    head = hdr.serialize(act) + struct.pack("<Q", 7)
    for n in (2**64 - 1, 2**32, 1_000_001, 3):
        t0 = time.time()
        with pytest.raises(ValueError):
            CompactBlock.from_payload(head + _ser_compact(n) + b"\x00" * 12, act)
        assert time.time() - t0 < 1.0
    with pytest.raises(ValueError):
        parse_getblocktxn(b"\x01" * 32 + _ser_compact(2**40) + b"\x00")
    with pytest.raises(ValueError):
        parse_getblocktxn(getblocktxn_payload(b"\x01" * 32, [0, 70000]))
    with pytest.raises(ValueError):
        parse_blocktxn(b"\x01" * 32 + _ser_compact(2**63))


def _handshake(port, magic):
    sock = socket.create_connection(("127.0.0.1", port))
    sock.sendall(P.frame(magic, "version", P.version_payload(0, nonce=42)))
    seen = set()
    while not {"version", "verack"} <= seen:
        cmd, _ = P.read_message(sock, magic)
        seen.add(cmd)
    sock.sendall(P.frame(magic, "verack"))
    return sock


def _read_until(sock, magic, want, timeout=20.0):
    sock.settimeout(timeout)
    while True:
        cmd, payload = P.read_message(sock, magic)
        if cmd == want:
            return payload


def test_compact_block_relay_between_nodes(core, tmp_path):
    a = _node(core, tmp_path, "a", ["-listen", "-port=0"])
    b = None
    try:
        w = a.wallet.new_address()
        wspk = core.address_to_script(w, a.params.pubkey_prefix, a.params.script_prefix)
        a.miner.generate(wspk, 101)
        b = _node(core, tmp_path, "b", [f"-connect=127.0.0.1:{a.connman.port}"])
        assert _wait(lambda: b.state.height() == 101 and b.peer_count() == 1)
        # b asks a for high-bandwidth compact blocks
        b.connman.peers[0].send("sendcmpct", struct.pack("<?Q", True, 2))
        assert _wait(lambda: a.connman.peers and a.connman.peers[0].cmpct_hb)
        txid = a.wallet.send([(b"\x51", 10**8)])
        assert _wait(lambda: txid in b.state.mempool)
        before = REGISTRY.total("p2p_cmpct_reconstructed_total")
        asked = REGISTRY.total("p2p_cmpct_getblocktxn_total")
        a.miner.generate(a.mining_script, 1)
        assert _wait(lambda: b.state.coins_tip().hash == a.state.tip().hash and txid not in b.state.mempool)
        # rebuilt from b's own mempool: no getblocktxn round trip
        assert REGISTRY.total("p2p_cmpct_reconstructed_total") > before
        assert REGISTRY.total("p2p_cmpct_getblocktxn_total") == asked
    finally:
        if b is not None:
            b.stop()
        a.stop()


def test_bloom_merkleblock_and_getaddr(core, tmp_path):
    a = _node(core, tmp_path, "a", ["-listen", "-port=0"])
    try:
        w = a.wallet.new_address()
        wspk = core.address_to_script(w, a.params.pubkey_prefix, a.params.script_prefix)
        a.miner.generate(wspk, 101)
        dest_h = bytes(range(40, 60))  # not the test nodes' mining address (bytes(range(20)))
        txid = a.wallet.send([(b"\x76\xa9\x14" + dest_h + b"\x88\xac", 2 * 10**8)])
        bh = a.miner.generate(a.mining_script, 1)[0]
        magic = bytes(a.params.message_start)
        sock = _handshake(a.connman.port, magic)
        f = BloomFilter.create(10, 0.0001, 5, BLOOM_UPDATE_ALL)
        f.insert(dest_h)
        sock.sendall(P.frame(magic, "filterload", f.payload()))
        sock.sendall(P.frame(magic, "getdata", P.inv_payload([(3, core.u256_from_hex(bh))])))
        mb = _read_until(sock, magic, "merkleblock")
        tx = _read_until(sock, magic, "tx")
        assert core.Transaction.deserialize(tx).txid() == txid
        hdr, used = core.BlockHeader.deserialize_prefix(mb, a.params.kawpow_activation_time, 0)
        assert a.state.block_hash(hdr) == core.u256_from_hex(bh)
        assert struct.unpack_from("<I", mb, used)[0] == 2  # the partial tree covers both transactions
        # getaddr from an inbound peer is answered once from the address manager
        now = int(time.time())
        a.connman.addrman.add([("198.51.100.7", 8788, 1, now - 100), ("198.51.100.8", 8788, 1, now - 100)], "127.0.0.1")
        sock.sendall(P.frame(magic, "getaddr"))
        got = _parse_addr(_read_until(sock, magic, "addr"))
        assert got and all(ip.startswith("198.51.100.") for ip, _, _, _ in got)
        sock.close()
    finally:
        a.stop()


def test_compact_block_uses_extra_txn(core, tmp_path):
    """-blockreconstructionextratxn (vExtraTxnForCompact): a transaction b saw but no longer holds
    in its mempool (rejected, orphaned or replaced) still fills its slot of a compact block."""
    a = _node(core, tmp_path, "a", ["-listen", "-port=0"])
    b = None
    try:
        w = a.wallet.new_address()
        wspk = core.address_to_script(w, a.params.pubkey_prefix, a.params.script_prefix)
        a.miner.generate(wspk, 101)
        b = _node(core, tmp_path, "b", [f"-connect=127.0.0.1:{a.connman.port}", "-blockreconstructionextratxn=10"])
        assert b.connman.extra_txn.maxlen == 10
        assert _wait(lambda: b.state.height() == 101 and b.peer_count() == 1)
        b.connman.peers[0].send("sendcmpct", struct.pack("<?Q", True, 2))
        assert _wait(lambda: a.connman.peers and a.connman.peers[0].cmpct_hb)
        txid = a.wallet.send([(b"\x51", 10**8)])
        assert _wait(lambda: txid in b.state.mempool)
        with b.state.lock:
            tx = b.state.mempool[txid].tx
            b.state.pool_remove(txid)
        b.connman.extra_txn.append(tx)
        asked = REGISTRY.total("p2p_cmpct_getblocktxn_total")
        a.miner.generate(a.mining_script, 1)
        assert _wait(lambda: b.state.coins_tip().hash == a.state.tip().hash)
        assert REGISTRY.total("p2p_cmpct_getblocktxn_total") == asked  # no round trip for it
    finally:
        if b is not None:
            b.stop()
        a.stop()
