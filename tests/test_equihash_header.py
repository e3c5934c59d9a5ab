"""Equihash(200,9) header extension (new): format,
consensus checks, DGW era bootstrap, batch verification — CPU paths.
The reference has no Equihash, so parity is "unpinned"; the rules are pinned
against the CPU golden verifier (csrc/pow/equihash.cpp) instead."""
import pytest


@pytest.fixture(scope="module")
def mixed_chain():
    from nodexa_chain_core_amd.models import synthetic

    # regtest limit 2^255: ~2 hashes / ~1 solve per header keeps the CPU mining short
    return synthetic.build_chain(3, 2, network="regtest", seed=7)


def test_format_roundtrip_and_flag(core, mixed_chain):
    params, headers = mixed_chain
    act = params.kawpow_activation_time
    kp, eq = headers[0], headers[-1]
    assert not kp.is_equihash() and eq.is_equihash()
    assert len(kp.serialize(act)) == 120
    raw = eq.serialize(act)
    assert len(raw) == 80 + 32 + 3 + 1344  # prefix | nonce256 | CompactSize(1344) | solution
    back = core.BlockHeader.deserialize(raw, act)
    assert back.serialize(act) == raw and back.solution == eq.solution and back.nonce256 == eq.nonce256
    assert eq.equihash_input() == eq.kawpow_input() + eq.nonce256
    # block hash = SHA256d(serialized header)
    assert eq.equihash_hash(act) == core.sha256d(raw)
    both = core.deserialize_headers(b"".join(h.serialize(act) for h in headers), act)
    assert [h.serialize(act) for h in both] == [h.serialize(act) for h in headers]


def test_chain_accepts_and_rejects(core, mixed_chain):
    params, headers = mixed_chain
    act = params.kawpow_activation_time
    chain = core.HeaderChain(params)
    adj = headers[-1].time + 60
    for h in headers[:-1]:
        assert chain.accept_header(h, adj, True).ok
    last = headers[-1]
    # corrupted solution -> invalid-solution
    bad = core.BlockHeader.deserialize(last.serialize(act), act)
    sol = bytearray(bad.solution)
    sol[100] ^= 0x40
    bad.solution = bytes(sol)
    assert chain.accept_header(bad, adj, True).reject == "invalid-solution"
    # truncated solution
    bad.solution = bytes(last.solution[:-1])
    assert chain.accept_header(bad, adj, True).reject == "invalid-solution"
    # a KawPow-format header inside the Equihash era
    kp = core.BlockHeader.deserialize(last.serialize(act), act)
    kp.version &= ~core.EQUIHASH_VERSION_BIT
    assert chain.accept_header(kp, adj, False).reject == "bad-version(equihash-required)"
    # wrong committed height
    wh = core.BlockHeader.deserialize(last.serialize(act), act)
    wh.height += 1
    r = chain.accept_header(wh, adj, False)
    assert r.reject == "bad-height"
    assert chain.accept_header(last, adj, True).ok and chain.height() == len(headers)


def test_flag_forbidden_before_activation(core, mixed_chain):
    params, headers = mixed_chain
    act = params.kawpow_activation_time
    chain = core.HeaderChain(params)
    h = core.BlockHeader.deserialize(headers[0].serialize(act), act)
    h.version |= core.EQUIHASH_VERSION_BIT
    h.nonce256 = bytes(32)
    h.solution = bytes(1344)
    assert chain.accept_header(h, h.time + 60, False).reject == "bad-version(equihash-not-active)"


def test_dgw_bootstraps_equihash_era(core):
    from nodexa_chain_core_amd.chain.state import make_params

    p = make_params("test", kawpow_activation_time=1, equihash_activation_time=1)
    assert p.equihash_limit == bytes(32)  # null -> pow limit
    lim = bytes.fromhex("000fffff" + "ff" * 28)[::-1]  # 2^236-ish, storage order
    p.equihash_limit = lim
    chain = core.HeaderChain(p)
    g = chain.tip()
    # fewer than 180 blocks: DGW's early return gives pow limit; the era rule kicks in
    # once the window is full but not yet all Equihash — checked via the C++ DGW directly
    h = core.BlockHeader()
    h.time = g.time + 60
    assert chain.next_bits(h) == 0x2000ffff  # < 180 blocks -> testnet pow limit compact


def test_batch_verify_cpu(core, mixed_chain):
    from nodexa_chain_core_amd.models.verify import verify_headers

    params, headers = mixed_chain
    act = params.kawpow_activation_time
    res = verify_headers(params, headers, gpus=None)
    assert all(r["valid"] for r in res), res
    bad = core.BlockHeader.deserialize(headers[-1].serialize(act), act)
    sol = bytearray(bad.solution)
    sol[7] ^= 1
    bad.solution = bytes(sol)
    assert verify_headers(params, [bad], gpus=None)[0]["reason"] == "invalid-solution"


@pytest.mark.parametrize("name", ["testnet_kawpow_10k.hdr", "testnet_mixed_10k.hdr"])
def test_synthetic_fixture_chain(core, name):
    """The committed BASELINE config-5 fixtures (GPU-mined): every header passes the
    contextual rules and DGW in a fresh header chain; PoW is checked on CPU for a sample
    of KawPow headers and for every Equihash-extension header."""
    import os

    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import verify_headers

    params, headers = synthetic.load(os.path.join(os.path.dirname(__file__), "data", name))
    assert len(headers) == 10000
    chain = core.HeaderChain(params)
    for h in headers:
        r = chain.accept_header(h, headers[-1].time + 3600, False)
        assert r.ok, r.reject
    eq = [h for h in headers if h.is_equihash()]
    assert len(eq) == (170 if "mixed" in name else 0)
    sample = headers[:40] + headers[7490:7510] + eq
    res = verify_headers(params, sample)
    assert all(r["valid"] for r in res), [r for r in res if not r["valid"]][:3]


def test_resident_path_declines_malformed_equihash(core, mixed_chain):
    """a peer's `headers` batch with one Equihash header whose solution is not 1344 bytes
    must not reach the resident pipeline (it would raise and drop the peer unscored); the resident
    entry declines it (None), and process_headers keeps the valid prefix and rejects the bad
    header as invalid-solution (the DoS-100 rule of net/p2p.on_headers)."""
    from nodexa_chain_core_amd.models.verify import process_batch_resident, process_headers

    params, headers = mixed_chain
    act = params.kawpow_activation_time
    last = headers[-1]
    bad = core.BlockHeader.deserialize(last.serialize(act), act)
    bad.solution = bytes(last.solution[:-1])
    batch_headers = list(headers[:-1]) + [bad]
    batch = core.HeaderBatch.from_headers(batch_headers, act)
    assert not batch.eq_uniform
    chain = core.HeaderChain(params)
    assert process_batch_resident(chain, batch, last.time + 60, device=0) is None  # no GPU touched
    res = process_headers(chain, batch_headers, last.time + 60, gpus=None)
    assert res["accepted"] == len(headers) - 1
    assert res["reject"]["reason"] == "invalid-solution"
