"""Consensus layer (csrc/chain/*) vs reference fixtures and independent oracles."""
import os
import struct

import pytest

# Subsidy values the reference pins in its Windows libm patch table
# (src/validation.cpp:1345-8975) — i.e. the Linux pow() results.
SUBSIDY_PINS = [(76084, 52501147075), (78768, 52442437565), (1289307, 31660802101), (2052805, 23030061450),
                (2685026, 17694374225), (3431098, 12964723721), (4202212, 9400644252), (5025499, 6669700849),
                (6176325, 4128155857), (7779336, 2116120452), (10774335, 607174402), (19482328, 16098395),
                (19861632, 13743958), (20797544, 9304016), (25932669, 1093921)]


def test_genesis_main(core):
    p = core.make_chain_params("main")
    g = p.genesis
    mr, mutated = g.merkle_root()
    # src/chainparams.cpp:180-181
    assert core.u256_hex(mr) == "7c1d71731b98c560a80cee3b88993c8c863342b9661894304fd843bf7e75a41f"
    assert not mutated
    h = core.x16r(g.header.legacy80(), g.header.prev)
    assert core.u256_hex(h) == "0000000a50fdaaf22f1c98b8c61559e15ab2269249aa1fb20683180703cdbf07"
    assert core.check_proof_of_work(h, g.header.bits, p)
    raw = g.serialize(p.kawpow_activation_time)
    assert len(raw) > 80 and raw[:4] == struct.pack("<i", 4)
    g2 = core.Block.deserialize(raw, p.kawpow_activation_time)
    assert g2.serialize(p.kawpow_activation_time) == raw


def test_genesis_regtest_and_chain(core):
    p = core.make_chain_params("regtest")
    chain = core.HeaderChain(p)
    assert chain.height() == 0
    g = chain.genesis()
    assert g.hash == core.x16r(p.genesis.header.legacy80(), bytes(32))
    assert chain.tip().hash == g.hash


def test_compact_roundtrip(core):
    for bits in [0x1d00ffff, 0x1e00ffff, 0x207fffff, 0x1b0404cb, 0x05009234, 0x04923456, 0x03123456]:
        v, neg, ovf = core.set_compact(bits)
        assert not ovf
        if not neg:
            assert core.get_compact(v) == bits or core.set_compact(core.get_compact(v))[0] == v
    v, neg, ovf = core.set_compact(0x01fedcba)
    assert neg and v == 0x7e
    v, neg, ovf = core.set_compact(0xff123456)
    assert ovf
    assert core.get_compact(0x80) == 0x02008000


def test_block_proof_and_difficulty(core):
    assert core.block_proof(0x207fffff) == 2
    assert core.difficulty_from_bits(0x1d00ffff) == pytest.approx(1.0)
    assert core.difficulty_from_bits(0x1e00ffff) == pytest.approx(1 / 256)


def test_subsidy_pins(core):
    assert core.block_subsidy(0) == 54193019856
    for h, v in SUBSIDY_PINS:
        assert core.block_subsidy(h) == v, h


def test_script_and_addresses(core):
    p = core.make_chain_params("main")
    spk = core.address_to_script(p.community_autonomous_address, p.pubkey_prefix, p.script_prefix)
    assert spk is not None and len(spk) == 25 and spk[:3] == b"\x76\xa9\x14"
    assert core.script_to_address(spk, p.pubkey_prefix, p.script_prefix) == p.community_autonomous_address
    assert core.address_to_script(p.community_autonomous_address, 42, 124) is None  # wrong network
    assert core.script_push_int(5) == b"\x55"
    assert core.script_push_int(0) == b"\x00"
    assert core.script_push_int(200) == b"\x02\xc8\x00"
    assert core.scriptnum(-1) == b"\x81"
    assert core.ripemd160(b"").hex() == "9c1185a5c5e9fc54612808977ee8f548b2258d31"


def _oracle_dgw(headers, next_time, pow_limit, kawpow_limit, act, spacing=60):
    """Independent Python DarkGravityWave (semantics of src/pow.cpp:18-102, non-regtest)."""
    def set_compact(bits):
        size, word = bits >> 24, bits & 0x7FFFFF
        return word >> 8 * (3 - size) if size <= 3 else word << 8 * (size - 3)

    def get_compact(v):
        size = (v.bit_length() + 7) // 8
        c = (v << 8 * (3 - size)) if size <= 3 else (v >> 8 * (size - 3))
        c &= 0xFFFFFFFF
        if c & 0x00800000:
            c >>= 8
            size += 1
        return c | (size << 24)

    M = (1 << 256) - 1
    last_h = len(headers) - 1
    if last_h < 180:
        return get_compact(pow_limit)
    avg = 0
    kaw = 0
    for n in range(1, 181):
        t, bits = headers[-n]
        tgt = set_compact(bits)
        avg = tgt if n == 1 else ((avg * n + tgt) & M) // (n + 1)
        kaw += t >= act
    if next_time >= act and kaw != 180:
        return get_compact(kawpow_limit)
    actual = headers[-1][0] - headers[-180][0]
    T = 180 * spacing
    actual = max(T // 3, min(3 * T, actual))
    new = ((avg * (actual & 0xFFFFFFFF)) & M) // T
    return get_compact(min(new, pow_limit))


@pytest.mark.parametrize("pattern", ["steady", "fast", "slow", "kawpow_switch"])
def test_dgw_against_oracle(core, pattern):
    p = core.make_chain_params("test")  # mainnet DGW rules, no checkpoints
    chain = core.HeaderChain(p)
    if pattern == "kawpow_switch" and not all(core.x16r_slot_available(a) for a in range(16)):
        pytest.skip("pre-KawPow headers need every X16R primitive")
    if pattern == "kawpow_switch":
        act = p.genesis.header.time + 150 * 60
    else:
        act = p.genesis.header.time  # every block after genesis is KawPow-time
    chain.set_kawpow_activation_time(act)
    pow_limit = int.from_bytes(p.pow_limit[::-1], "big")
    gaps = {"steady": [60], "fast": [20, 25, 30], "slow": [200, 90, 400], "kawpow_switch": [55, 65]}[pattern]
    seq = [(p.genesis.header.time, p.genesis.header.bits)]
    prev = chain.tip()
    t = p.genesis.header.time
    for h in range(1, 420):
        t += gaps[h % len(gaps)]
        hdr = core.BlockHeader()
        hdr.version = 0x30000000
        hdr.prev = prev.hash
        hdr.merkle_root = core.sha256d(struct.pack("<I", h))
        hdr.time = t
        hdr.height = h
        hdr.bits = chain.next_bits(hdr)
        expect = _oracle_dgw(seq, t, pow_limit, pow_limit, chain.params.kawpow_activation_time)
        assert hdr.bits == expect, (h, hex(hdr.bits), hex(expect))
        r = chain.accept_header(hdr, t + 10, False)
        assert r.ok, r.reject
        prev = r.index
        seq.append((t, hdr.bits))
    assert chain.height() == 419


def test_contextual_rejections(core):
    p = core.make_chain_params("regtest")
    chain = core.HeaderChain(p)
    chain.set_kawpow_activation_time(0)
    g = chain.tip()
    hdr = core.BlockHeader()
    hdr.version = 0x30000000
    hdr.prev = g.hash
    hdr.time = g.time + 60
    hdr.height = 1
    hdr.bits = 0x1d00ffff
    assert chain.accept_header(hdr, hdr.time, False).reject == "bad-diffbits"
    hdr.bits = chain.next_bits(hdr)
    old = hdr.version
    hdr.version = 4
    assert chain.accept_header(hdr, hdr.time, False).reject.startswith("bad-version")
    hdr.version = old
    assert chain.accept_header(hdr, hdr.time - 3 * 3600, False).reject == "time-too-new"
    hdr.prev = b"\x11" * 32
    assert chain.accept_header(hdr, hdr.time, False).reject == "prev-blk-not-found"


def test_kawpow_header_full_check(core):
    """Mine a regtest KawPow header on the CPU (regtest target ~1/2) and run it
    through CheckBlockHeader's full path (light-mode KawPow + mix compare)."""
    p = core.make_chain_params("regtest")
    chain = core.HeaderChain(p)
    chain.set_kawpow_activation_time(0)
    g = chain.tip()
    hdr = core.BlockHeader()
    hdr.version = 0x30000000
    hdr.prev = g.hash
    hdr.time = g.time + 61
    hdr.height = 1
    hdr.bits = chain.next_bits(hdr)
    for nonce in range(64):
        hdr.nonce64 = nonce
        pow_hash, mix = chain.block_hash_full(hdr)
        if core.check_proof_of_work(pow_hash, hdr.bits, chain.params):
            hdr.mix_hash = mix
            break
    else:
        pytest.fail("no regtest KawPow solution in 64 nonces")
    assert chain.block_hash(hdr) == pow_hash  # mix-only hash == full hash when mix matches
    bad = core.BlockHeader.deserialize(hdr.serialize(0), 0)
    bad.mix_hash = bytes(32)
    assert not chain.check_header(bad, True).ok
    r = chain.accept_header(hdr, hdr.time, True)
    assert r.ok and chain.height() == 1


def test_blockstore_roundtrip(core, tmp_path):
    p = core.make_chain_params("regtest")
    st = core.BlockStore(str(tmp_path / "blocks"), p.message_start, p.kawpow_activation_time)
    g = p.genesis
    pos = st.write(g)
    pos2 = st.write(g)
    assert pos2.offset == pos.offset + pos.size + 8
    assert st.read(pos).serialize(p.kawpow_activation_time) == g.serialize(p.kawpow_activation_time)
    raw = open(st.path(0), "rb").read()
    assert raw[:4] == p.message_start == b"DROW"
    assert struct.unpack("<I", raw[4:8])[0] == pos.size
    assert len(st.scan()) == 2
    st2 = core.BlockStore(str(tmp_path / "blocks"), p.message_start, p.kawpow_activation_time)
    pos3 = st2.write(g)
    assert pos3.offset == pos2.offset + pos2.size + 8


def _fake_header(core, chain, prev, h, t, salt=0):
    hdr = core.BlockHeader()
    hdr.version = 0x30000000
    hdr.prev = prev.hash
    hdr.merkle_root = core.sha256d(struct.pack("<II", h, salt))
    hdr.time = t
    hdr.height = h
    hdr.bits = chain.next_bits(hdr) if prev.hash == chain.tip().hash else 0
    return hdr


def test_header_acceptance_scales_linearly(core):
    """ProcessNewBlockHeaders over 20k headers (PoW skipped): the active-chain update is
    incremental (fork depth), not a rescan of the whole index per header."""
    import time

    p = core.make_chain_params("test")
    chain = core.HeaderChain(p)
    chain.set_kawpow_activation_time(p.genesis.header.time)
    prev, t = chain.tip(), p.genesis.header.time
    t0 = time.perf_counter()
    for h in range(1, 20001):
        t += 61
        r = chain.accept_header(_fake_header(core, chain, prev, h, t), t + 10, False)
        assert r.ok, (h, r.reject)
        prev = r.index
    assert chain.height() == 20000
    assert time.perf_counter() - t0 < 10.0


def test_reorg_invalidate_reconsider(core):
    """A heavier side branch takes over; invalidating its first block falls back to the
    main branch (descendants excluded too); reconsider restores it."""
    p = core.make_chain_params("regtest")
    chain = core.HeaderChain(p)
    chain.set_kawpow_activation_time(p.genesis.header.time)
    g, t = chain.tip(), p.genesis.header.time
    main = [g]
    for h in range(1, 6):
        hdr = _fake_header(core, chain, main[-1], h, t + 60 * h)
        main.append(chain.accept_header(hdr, hdr.time + 10, False).index)
    # side branch from height 2, one block longer (same bits on regtest -> more work)
    side = [main[2]]
    for h in range(3, 8):
        hdr = _fake_header(core, chain, side[-1], h, t + 60 * h + 1, salt=1)
        hdr.bits = main[1].bits
        r = chain.accept_header(hdr, hdr.time + 10, False)
        assert r.ok, r.reject
        side.append(r.index)
    assert chain.tip().hash == side[-1].hash and chain.height() == 7
    assert chain.at_height(3).hash == side[1].hash
    chain.invalidate(side[1].hash)
    assert chain.tip().hash == main[-1].hash and chain.height() == 5
    chain.reconsider(side[1].hash)
    assert chain.tip().hash == side[-1].hash
