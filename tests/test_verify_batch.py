"""Batch header verification on the host (models/verify.py native path, no GPU).

Mirrors the reference's CheckBlockHeader outcomes (src/validation.cpp:11638-11665):
a header whose claimed mix cannot meet nBits is "high-hash" before any DAG work,
one whose claimed mix is wrong is "invalid-mix-hash", and ProcessNewBlockHeaders
stops at the first invalid header of a batch (src/validation.cpp:12017-12035).
"""
import os

import numpy as np
import pytest

from nodexa_chain_core_amd import core
from nodexa_chain_core_amd.chain.header import BlockHeader as PyHeader
from nodexa_chain_core_amd.models import synthetic
from nodexa_chain_core_amd.models.verify import _rows_le, process_headers, verify_headers

_core = core()
FIX = os.path.join(os.path.dirname(__file__), "data", "testnet_kawpow_10k.hdr")


@pytest.fixture(scope="module")
def chain_fixture():
    return synthetic.load(FIX)


def _copy(h, act):
    return _core.BlockHeader.deserialize(h.serialize(act), act)


def test_rows_le_matches_hash_le():
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    b = a.copy()
    b[50:] = rng.integers(0, 256, (150, 32), dtype=np.uint8)
    b[100:150, :20] = a[100:150, :20]  # long common prefixes
    got = _rows_le(a, b)
    want = [_core.hash_le(x.tobytes(), y.tobytes()) for x, y in zip(a, b)]
    assert got.tolist() == want


def test_valid_prefix_and_hashes(chain_fixture):
    params, headers = chain_fixture
    act = params.kawpow_activation_time
    res = verify_headers(params, headers[:24], threads=4)
    assert all(r["valid"] for r in res)
    for h, r in zip(headers[:24], res):  # hash == KAWPOWHash (block hash), light context
        ctx = _core.get_epoch_context(h.height // _core.EPOCH_LENGTH)
        fin, _ = _core.kawpow_hash(ctx, h.height, h.kawpow_header_hash()[::-1], h.nonce64)
        assert r["hash"] == fin.hex()
    # Python dataclass headers take the same path
    py = [PyHeader.deserialize(h.serialize(act), act)[0] for h in headers[:4]]
    assert verify_headers(params, py, threads=2) == res[:4]


def test_invalid_mix_and_high_hash(chain_fixture):
    params, headers = chain_fixture
    act = params.kawpow_activation_time
    base = headers[10]
    # wrong nonce64 with the original mix: either the mix-only prefilter already fails
    # (high-hash) or the recomputed mix differs (invalid-mix-hash) — find one of each.
    seen = {}
    for d in range(1, 400):
        h = _copy(base, act)
        h.nonce64 = base.nonce64 + d
        r = verify_headers(params, [h], threads=1)[0]
        assert not r["valid"]
        seen.setdefault(r["reason"], d)
        if len(seen) == 2:
            break
    assert set(seen) == {"high-hash", "invalid-mix-hash"}


def test_process_headers_stops_at_first_invalid(chain_fixture):
    params, headers = chain_fixture
    act = params.kawpow_activation_time
    batch = [_copy(h, act) for h in headers[:20]]
    bad = batch[12]
    bad.mix_hash = bytes(32)
    chain = _core.HeaderChain(params)
    r = process_headers(chain, batch, headers[-1].time + 3600)
    assert r["accepted"] == 12 and r["reject"]["index"] == 12
    assert r["reject"]["reason"] in ("high-hash", "invalid-mix-hash")
    assert chain.height() == 12
    # a contextual failure (here: an unconnected header) is reported at its index
    chain = _core.HeaderChain(params)
    batch = [_copy(h, act) for h in headers[:5] + headers[6:9]]
    r = process_headers(chain, batch, headers[-1].time + 3600)
    assert r["accepted"] == 5 and r["reject"]["index"] == 5 and chain.height() == 5


def test_arith_div_matches_python_ints():
    import random

    rng = random.Random(7)
    for _ in range(5000):
        a = rng.getrandbits(rng.randint(1, 256))
        b = rng.getrandbits(rng.randint(1, 256)) or 1
        assert _core.arith_div(a, b) == a // b


@pytest.mark.parametrize("fixture", ["testnet_kawpow_10k.hdr", "testnet_mixed_10k.hdr"])
def test_accept_headers_batch_equals_serial(fixture):
    """accept_headers precomputes hashes + DGW for a linear batch on all cores; results,
    tip and chain work must equal header-by-header acceptance (incl. the Equihash
    bootstrap and DGW overflow eras of the mixed fixture)."""
    params, headers = synthetic.load(os.path.join(os.path.dirname(__file__), "data", fixture))
    act = params.kawpow_activation_time
    adj = headers[-1].time + 3600
    a = _core.HeaderChain(params)
    ra = a.accept_headers(list(headers), adj, False)
    b = _core.HeaderChain(params)
    rb = [b.accept_header(h, adj, False) for h in headers]
    assert [r.ok for r in ra] == [r.ok for r in rb] == [True] * len(headers)
    assert a.tip().hash == b.tip().hash and a.tip().chain_work == b.tip().chain_work
    # a wrong nBits in the middle: same reject at the same index, earlier headers kept
    bad = list(headers)
    h = _copy(headers[5000], act)
    h.bits ^= 1
    bad[5000] = h
    c = _core.HeaderChain(params)
    rc = c.accept_headers(bad, adj, False)
    assert len(rc) == 5001 and rc[-1].reject == "bad-diffbits" and c.height() == headers[4999].height
    # full PoW checked in parallel (check_pow=True) accepts the valid prefix
    d = _core.HeaderChain(params)
    assert all(r.ok for r in d.accept_headers(list(headers[:96]), adj, True))
    # the batch's median-time-past comes from its own time series: a last header at (or below)
    # its parent's MTP is refused as one by one (the batch stays linear: nothing follows it)
    for cut in (12, 3000):
        hs = list(headers[:cut])
        e = _core.HeaderChain(params)
        assert all(r.ok for r in e.accept_headers(hs[:-1], adj, False))
        mtp = e.tip().median_time_past()
        late = _copy(hs[-1], act)
        late.time = mtp
        f = _core.HeaderChain(params)
        rf = f.accept_headers(hs[:-1] + [late], adj, False)
        assert len(rf) == cut and rf[-1].reject == "time-too-old", (cut, rf[-1].reject)


def test_accept_headers_with_precomputed_hashes_and_bits():
    """The batch path's inputs from the PoW stage / GPU: block hashes and the DGW nBits of each
    header (`dgw_series` is the series the GPU kernel reads). Correct values give the same chain;
    a wrong expected nBits is a bad-diffbits reject at that header; 0 leaves it to the host."""
    import struct

    params, headers = synthetic.load(os.path.join(os.path.dirname(__file__), "data", "testnet_mixed_10k.hdr"))
    hs = list(headers[:3000])
    adj = headers[-1].time + 3600
    ref = _core.HeaderChain(params)
    assert all(r.ok for r in ref.accept_headers(hs, adj, False))
    hashes = b"".join(ref.block_hash(h) for h in hs)
    fresh = _core.HeaderChain(params)
    times, bits, a, base = fresh.dgw_series(hs, hashes)
    assert a == 1 and base == 0 and len(times) == len(bits) == 4 * (a + len(hs))
    assert struct.unpack_from("<I", bits, 4 * (a + 7))[0] == hs[7].bits
    want = b"".join(struct.pack("<I", h.bits) for h in hs)  # a valid chain carries its expected nBits
    r = fresh.accept_headers(hs, adj, False, hashes, want)
    assert all(x.ok for x in r) and fresh.tip().hash == ref.tip().hash
    wrong = bytearray(want)
    struct.pack_into("<I", wrong, 4 * 1500, hs[1500].bits ^ 1)
    c = _core.HeaderChain(params)
    rc = c.accept_headers(hs, adj, False, hashes, bytes(wrong))
    assert len(rc) == 1501 and rc[-1].reject == "bad-diffbits"
    zeros = _core.HeaderChain(params)
    assert all(x.ok for x in zeros.accept_headers(hs, adj, False, hashes, bytes(4 * len(hs))))
    with pytest.raises(ValueError):
        _core.HeaderChain(params).accept_headers(hs, adj, False, hashes[:-1])


def test_max_reorg_depth_guard(chain_fixture):
    """-maxreorg (ContextualCheckBlockHeader): with the guard armed a fork from >= 60 blocks
    below the tip is rejected with DoS 10; disarmed it is stored as a side branch."""
    params, headers = chain_fixture
    act = params.kawpow_activation_time
    adj = headers[-1].time + 3600
    chain = _core.HeaderChain(params)
    assert all(r.ok for r in chain.accept_headers(list(headers[:100]), adj, False))
    tip = chain.tip().hash
    fork = _copy(headers[20], act)  # same parent (height 20), different nonce: a new branch
    fork.nonce64 ^= 1
    deep = chain.height() - headers[19].height
    assert deep >= params.max_reorg_depth == 60
    chain.max_reorg_depth = params.max_reorg_depth
    r = chain.accept_header(fork, adj, False)
    assert not r.ok and r.reject == "bad-fork-prior-to-maxreorgdepth" and r.dos == 10
    shallow = _copy(headers[95], act)  # 5 below the tip: allowed even when armed
    shallow.nonce64 ^= 1
    assert chain.accept_header(shallow, adj, False).ok
    chain.max_reorg_depth = 0
    assert chain.accept_header(fork, adj, False).ok and chain.tip().hash == tip


def test_header_batch_rows_and_accept_batch(core):
    """csrc/chain/headerbatch.hpp: parsed from the wire bytes in parallel, packed rows equal the
    serializations, and HeaderChain.accept_batch over [lo, hi) ranges builds the same chain as
    accept_headers (hashes / nBits omitted: computed on the host)."""
    import os

    import numpy as np

    from nodexa_chain_core_amd.models import synthetic

    path = os.path.join(os.path.dirname(__file__), "data", "testnet_mixed_10k.hdr")
    params, hs = synthetic.load(path)
    act = params.kawpow_activation_time
    raw = open(path, "rb").read()
    b = core.HeaderBatch.from_bytes(raw, act)
    assert len(b) == len(hs) and b.eq_uniform and b.eq_ser_len == len(hs[-1].serialize(act))
    rows = np.frombuffer(b.rows, np.uint8).reshape(-1, 128)
    kinds = np.frombuffer(b.kinds, np.uint8)
    eq = np.frombuffer(b.eq_index, np.uint32)
    for i in (0, 1, 4999, int(eq[0]), len(hs) - 1):
        h = hs[i]
        if h.is_equihash():
            assert kinds[i] == 2 and rows[i, :80].tobytes() == h.kawpow_input()
        else:
            assert kinds[i] == 0 and rows[i, :120].tobytes() == h.serialize(act)
    k = list(eq).index(int(eq[0]))
    assert bytes(b.eq_sols)[k * 1344:(k + 1) * 1344] == hs[int(eq[0])].solution
    assert bytes(b.eq_msgs)[k * 128:k * 128 + 112] == hs[int(eq[0])].equihash_input()
    adj = hs[-1].time + 3600
    ref = core.HeaderChain(params)
    ref.accept_headers(list(hs[:3000]), adj, True)
    c = core.HeaderChain(params)
    assert c.accept_batch(b, adj, None, None, 0, 1500) == (1500, None, 0)
    assert c.accept_batch(b, adj, None, None, 1500, 3000) == (1500, None, 0)
    assert c.tip().hash == ref.tip().hash
    with pytest.raises(Exception):
        core.HeaderBatch.from_bytes(raw[:-7], act)  # truncated


def test_header_batch_wire_pack_equals_object_pack(core):
    """from_bytes packs rows / kinds / Equihash inputs, solutions and serializations straight from
    the wire records and decodes the header objects later (materialize): every packed byte equals
    from_headers' packing of the decoded objects, legacy 80-byte records included."""
    import os

    import numpy as np

    from nodexa_chain_core_amd.models import synthetic

    path = os.path.join(os.path.dirname(__file__), "data", "testnet_mixed_10k.hdr")
    params, hs = synthetic.load(path)
    act = params.kawpow_activation_time
    # a legacy (pre-KawPow) record in front: the same fields, 80-byte wire form
    leg = core.BlockHeader()
    leg.version, leg.prev, leg.merkle_root = 0x20000000, hs[0].prev, hs[0].merkle_root
    leg.time, leg.bits, leg.nonce = act - 60, hs[0].bits, 12345
    objs = [leg] + list(hs)
    raw = b"".join(h.serialize(act) for h in objs)
    a = core.HeaderBatch.from_bytes(raw, act)
    b = core.HeaderBatch.from_headers(objs, act)
    assert len(a) == len(b) == len(objs)
    for name in ("rows", "kinds", "eq_index", "eq_msgs", "eq_sols", "eq_ser"):
        assert bytes(getattr(a, name)) == bytes(getattr(b, name)), name
    assert (a.eq_ser_len, a.eq_uniform) == (b.eq_ser_len, b.eq_uniform)
    assert np.frombuffer(a.kinds, np.uint8)[0] == 3
    a.materialize()
    a.materialize()  # idempotent
    for i in (0, 1, 2, 5000, len(objs) - 1):
        assert a.header(i).serialize(act) == objs[i].serialize(act)
    # an accessor decodes on first use without an explicit materialize
    c = core.HeaderBatch.from_bytes(raw, act)
    assert [h.serialize(act) for h in c.headers(0, 3)] == [h.serialize(act) for h in objs[:3]]
    bad = bytearray(raw[80:80 + 120 * 3])
    with pytest.raises(Exception):
        core.HeaderBatch.from_bytes(bytes(bad[:-1]), act)
    # a mutable buffer is copied: changing it after the parse changes nothing the batch decodes
    buf = bytearray(raw)
    d = core.HeaderBatch.from_bytes(buf, act)
    buf[:] = bytes(len(buf))
    assert d.header(1).serialize(act) == objs[1].serialize(act)
    assert [h.serialize(act) for h in d.headers(5000, 5002)] == [h.serialize(act) for h in objs[5000:5002]]


def test_copy_into_is_bounded(core):
    """_core.copy_into (the resident verify's row staging): a parallel copy into a writable buffer
    at an offset, refusing anything that would not fit."""
    import numpy as np

    src = np.random.default_rng(1).integers(0, 256, 1 << 20, dtype=np.uint8)
    dst = np.zeros((1 << 20) + 4096, dtype=np.uint8)
    core.copy_into(dst, 4096, src)
    assert bytes(dst[4096:]) == src.tobytes() and not dst[:4096].any()
    small = np.zeros(16, dtype=np.uint8)
    core.copy_into(small, 8, b"abcdefgh")
    assert bytes(small[8:]) == b"abcdefgh"
    with pytest.raises(Exception):
        core.copy_into(small, 9, b"abcdefgh")
    with pytest.raises(Exception):
        core.copy_into(small, 17, b"")
    with pytest.raises(Exception):
        core.copy_into(b"read-only target", 0, b"x")
    # several parts in one call; nothing is written when any part does not fit
    big = np.zeros(1 << 21, dtype=np.uint8)
    core.copy_into_many(big, [(0, src), (1 << 20, b"xyz"), ((1 << 20) + 3, np.array([7, 8], np.uint32))])
    assert bytes(big[:1 << 20]) == src.tobytes() and bytes(big[(1 << 20):(1 << 20) + 11]) == b"xyz" + bytes([7, 0, 0, 0, 8, 0, 0, 0])
    clean = np.zeros(16, dtype=np.uint8)
    with pytest.raises(Exception):
        core.copy_into_many(clean, [(0, b"ok"), (15, b"too long")])
    assert not clean.any()


def test_prepare_commit_equals_accept(core):
    """HeaderChain.prepare_batch / commit_batch (the resident verify's two-phase accept): committing a
    prefix of a prepared batch builds the same chain as accept_batch over that prefix, and a chain
    changed between the two phases (another header accepted, a block invalidated) is prepared
    again rather than trusted."""
    import os

    import numpy as np

    from nodexa_chain_core_amd.models import synthetic

    path = os.path.join(os.path.dirname(__file__), "data", "testnet_mixed_10k.hdr")
    params, hs = synthetic.load(path)
    act = params.kawpow_activation_time
    raw = open(path, "rb").read()
    adj = hs[-1].time + 3600
    ref = core.HeaderChain(params)
    assert ref.accept_batch(core.HeaderBatch.from_bytes(raw, act), adj) == (len(hs), None, 0)
    n = len(hs)
    hashes = np.frombuffer(b"".join(ref.at_height(i + 1).hash for i in range(n)), np.uint8).reshape(n, 32).copy()
    bits = np.array([h.bits for h in hs], dtype="<u4")
    for hi in (n, 4321, 0):
        c = core.HeaderChain(params)
        b = core.HeaderBatch.from_bytes(raw, act)
        prep = c.prepare_batch(b, adj, hashes, bits)
        del b  # the prepared state keeps the batch alive
        assert c.commit_batch(prep, hi) == (hi, None, 0)
        assert c.height() == hi and c.tip().hash == (ref.at_height(hi).hash if hi else c.genesis().hash)
    # the chain moves between prepare and commit: the first 10 headers arrive on their own
    c = core.HeaderChain(params)
    b = core.HeaderBatch.from_bytes(raw, act)
    prep = c.prepare_batch(b, adj, hashes, bits)
    assert c.accept_batch(b, adj, None, None, 0, 10) == (10, None, 0)
    assert c.commit_batch(prep, 3000) == (3000, None, 0)  # the first 10 are duplicates now
    assert c.height() == 3000 and c.tip().hash == ref.at_height(3000).hash
    # a wrong nBits at 2500 (as the device would report it) stops the commit there
    bad = bits.copy()
    bad[2500] ^= 1
    c = core.HeaderChain(params)
    prep = c.prepare_batch(core.HeaderBatch.from_bytes(raw, act), adj, hashes, bad)
    acc, why, dos = c.commit_batch(prep, n)
    assert (acc, why) == (2500, "bad-diffbits") and c.height() == 2500
    with pytest.raises(ValueError):
        c.prepare_batch(core.HeaderBatch.from_bytes(raw, act), adj, hashes[:10], bits)


def test_kawpow_plan_matches_numpy(core):
    """HeaderBatch.kawpow_plan (the resident verify's plan in one native pass): the KawPow rows'
    epoch ranges and every row's nHeight / nTime / nBits, None for descending epochs."""
    import os

    import numpy as np

    from nodexa_chain_core_amd.models import synthetic

    path = os.path.join(os.path.dirname(__file__), "data", "testnet_mixed_10k.hdr")
    params, hs = synthetic.load(path)
    act = params.kawpow_activation_time
    b = core.HeaderBatch.from_bytes(open(path, "rb").read(), act)
    ranges, heights, times, bits = b.kawpow_plan(core.EPOCH_LENGTH)
    rows = np.frombuffer(b.rows, np.uint8).reshape(len(b), 128)
    kinds = np.frombuffer(b.kinds, np.uint8)
    kp = np.flatnonzero(kinds == 0)
    ep = np.ascontiguousarray(rows[kp, 76:80]).view("<u4").ravel() // core.EPOCH_LENGTH
    want = [(int(e), int(kp[ep == e][0]), int(kp[ep == e][-1]) + 1) for e in np.unique(ep).tolist()]
    assert [tuple(r) for r in ranges] == want and len(want) == 2
    for col, got in ((76, heights), (68, times), (72, bits)):
        assert np.array_equal(np.frombuffer(got, "<u4"), np.ascontiguousarray(rows[:, col:col + 4]).view("<u4").ravel())
    assert np.array_equal(np.frombuffer(times, "<u4"), [h.time for h in hs])
    # a batch whose KawPow epochs go backwards has no plan
    back = b"".join(h.serialize(act) for h in list(hs[7600:7610]) + list(hs[100:110]))
    assert core.HeaderBatch.from_bytes(back, act).kawpow_plan(core.EPOCH_LENGTH) is None


def _serial(params, headers, adj, check_pow=False, chain=None):
    c = chain or _core.HeaderChain(params)
    out = []
    for h in headers:
        r = c.accept_header(h, adj, check_pow)
        out.append((r.ok, r.reject, r.dos, r.duplicate))
        if not r.ok:
            break
    return c, out


def _results(rs):
    return [(r.ok, r.reject, r.dos, r.duplicate) for r in rs]


def _same_chain(a, b):
    assert a.height() == b.height() and a.size() == b.size()
    assert a.tip().hash == b.tip().hash and a.tip().chain_work == b.tip().chain_work
    for h in range(0, a.height() + 1, 97):  # skip pointers: ancestor walks agree everywhere
        x, y = a.at_height(h), b.at_height(h)
        assert x.hash == y.hash and x.skip_height == y.skip_height
        assert a.tip().ancestor(h).hash == x.hash


def test_accept_headers_fast_path_equals_serial(chain_fixture):
    """The linear-batch path of accept_headers (contextual rules on all cores, runs of new headers
    on top of the tip inserted in bulk) against header-by-header acceptance: the same results,
    reject reasons, DoS scores, duplicate flags and chain -- for a batch that overlaps headers
    already indexed, one that forks below the tip, and a corrupted header at random positions."""
    import random

    params, headers = chain_fixture
    act = params.kawpow_activation_time
    adj = headers[-1].time + 3600
    hs = list(headers[:4000])
    rng = random.Random(11)
    cases = [("clean", hs, 0)]
    for kind in ("bits", "time-old", "time-new", "version", "mix-pow"):
        pos = rng.randrange(200, len(hs))
        bad = list(hs)
        h = _copy(hs[pos], act)
        if kind == "bits":
            h.bits ^= 1
        elif kind == "time-old":
            h.time = hs[pos - 6].time - 1
        elif kind == "time-new":
            h.time = adj + 3 * 3600
        elif kind == "version":
            h.version = 0x20000000
        else:
            h.mix_hash = bytes(32)
        bad[pos] = h
        cases.append((kind, bad[: pos + 1 + rng.randrange(0, 50)], 0))
    cases.append(("overlap", hs, 1500))  # the first 1500 are indexed before the batch arrives
    for name, batch, pre in cases:
        for check_pow in (False, True) if name == "mix-pow" else (False,):
            a, b = _core.HeaderChain(params), _core.HeaderChain(params)
            if pre:
                assert all(r.ok for r in a.accept_headers(batch[:pre], adj, False))
                _serial(params, batch[:pre], adj, chain=b)
            ra = _results(a.accept_headers(batch, adj, check_pow))
            _, rb = _serial(params, batch, adj, check_pow, chain=b)
            assert ra == rb, (name, check_pow, ra[-1], rb[-1], len(ra), len(rb))
            _same_chain(a, b)
    # a batch that forks below the active tip: a side branch with less work, then more work
    a, b = _core.HeaderChain(params), _core.HeaderChain(params)
    assert all(r.ok for r in a.accept_headers(hs[:3000], adj, False))
    _serial(params, hs[:3000], adj, chain=b)
    fork = []
    for i in range(2500, 2500 + 700):
        h = _copy(hs[i], act)
        if i == 2500:
            h.nonce64 ^= 1
        else:
            h.prev = a.block_hash(fork[-1]) if fork else h.prev
        fork.append(h)
    ra = _results(a.accept_headers(fork, adj, False))
    _, rb = _serial(params, fork, adj, chain=b)
    assert ra == rb and all(r[0] for r in ra) and a.tip().hash == b.tip().hash
    assert a.tip().hash == a.block_hash(fork[-1]) and a.height() == hs[2500].height + 699
    _same_chain(a, b)


def test_wave_slots_group_rows_by_period():
    """ops/header_batch.wave_slots (kawpow_verify_waves' table): every KawPow row exactly once, the
    4 slots of a wave all of one ProgPoW period, slot 0 of a wave never idle, values relative to lo."""
    import numpy as np

    from nodexa_chain_core_amd.ops.header_batch import ResidentHeaderVerifier

    rng = np.random.default_rng(5)
    for _ in range(20):
        n = int(rng.integers(1, 400))
        heights = np.sort(rng.integers(7500, 7500 + 600, n)).astype(np.uint32)
        if rng.random() < 0.3:
            heights = rng.permutation(heights)  # arbitrary claimed heights: still grouped correctly
        lo = int(rng.integers(0, 5))
        idx = np.sort(rng.choice(np.arange(lo, n), size=int(rng.integers(1, max(2, n - lo))), replace=False)) \
            if n > lo else np.arange(0)
        slots = ResidentHeaderVerifier.wave_slots(idx, heights, lo)
        assert len(slots) % 4 == 0
        got = slots[slots >= 0] + lo
        assert sorted(got.tolist()) == sorted(idx.tolist())
        for w in slots.reshape(-1, 4):
            assert w[0] >= 0
            per = {int(heights[x + lo]) // 3 for x in w if x >= 0}
            assert len(per) == 1
        # the native table the resident pipeline uses (_core.wave_slots) is the same table
        kinds = np.full(n, 2, dtype=np.uint8)
        kinds[idx] = 0
        hi = int(idx[-1]) + 1 if len(idx) else lo
        assert (np.frombuffer(_core.wave_slots(kinds, heights, lo, hi), dtype=np.int32) == slots).all()


def test_resident_ready_policy(chain_fixture):
    """models/verify.resident_ready: P2P header batches take the device-resident path with
    -p2pverifymode=dag, or under "auto" once every epoch of the batch has a resident DAG on the
    device (a mining node's, shared through ops/verify.share_epoch) -- never by building a DAG for
    a 2000-header message."""
    from nodexa_chain_core_amd.models.verify import resident_ready
    from nodexa_chain_core_amd.ops import verify as V

    params, headers = chain_fixture
    act = params.kawpow_activation_time
    hs = list(headers[:2000])  # epoch 0
    assert resident_ready(hs, act, 0, "dag") and not resident_ready(hs, act, 0, "light")
    saved = dict(V._epochs)
    try:
        V._epochs.clear()
        assert not resident_ready(hs, act, 0, "auto")
        V.share_epoch(0, 0, object())
        assert resident_ready(hs, act, 0, "auto") and not resident_ready(hs, act, 1, "auto")
        assert not resident_ready(list(headers[7400:7600]), act, 0, "auto")  # spans epochs 0 and 1
    finally:
        V._epochs.clear()
        V._epochs.update(saved)


def test_workpool_exception_reaches_caller():
    """csrc/util/workpool.cpp: a part that throws (on a worker or on the caller) is rethrown on the
    caller after every part has returned, and the pool keeps working afterwards."""
    c = core()
    n = 100_000
    assert c.workpool_selftest(n) == n * (n - 1) // 2
    for bad in (0, n // 2, n - 1):
        with pytest.raises(RuntimeError, match="part failed"):
            c.workpool_selftest(n, bad)
        assert c.workpool_selftest(n) == n * (n - 1) // 2
