"""Equihash(200,9) CPU golden model (no reference implementation exists:
parity unpinned against the reference; checked against the public spec's
rules, RFC 7693 BLAKE2b and self-consistency)."""
import pytest


def test_blake2b_rfc7693(core):
    assert core.blake2b(b"abc").hex() == (
        "ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
        "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923")
    assert core.blake2b(b"").hex().startswith("786a02f742015903c6c6fd852552d272")


def test_params_200_9(core):
    p = core.EquihashParams(200, 9)
    assert p.collision_bits == 20
    assert p.num_leaves == 2 ** 21
    assert p.solution_indices == 512
    assert p.solution_bytes == 1344
    assert p.personal == b"ZcashPoW" + (200).to_bytes(4, "little") + (9).to_bytes(4, "little")


def test_pack_roundtrip(core):
    p = core.EquihashParams(200, 9)
    idx = [(i * 40961 + 7) % (1 << 21) for i in range(512)]
    packed = core.equihash_pack(p, idx)
    assert len(packed) == 1344
    assert core.equihash_unpack(p, packed) == idx


@pytest.fixture(scope="module")
def solved(core):
    p = core.EquihashParams(200, 9)
    for nonce in range(8):  # ~1.9 solutions per nonce on average; take the first that has one
        inp = bytes(80) + nonce.to_bytes(32, "little")
        sols, stats = core.equihash_solve_cpu(p, inp, 4, 8)
        if sols:
            break
    return p, inp, sols, stats


def test_solver_finds_valid_solutions(core, solved):
    p, inp, sols, stats = solved
    assert len(sols) >= 1, stats  # ~1.9 expected per nonce
    for s in sols:
        ok, why = core.equihash_verify(p, inp, s)
        assert ok, why
        assert len(set(s)) == 512


def test_verifier_rejections(core, solved):
    p, inp, sols, _ = solved
    s = list(sols[0])
    assert core.equihash_verify(p, inp + b"x", s)[0] is False
    bad = s[:]
    bad[0], bad[1] = bad[1], bad[0]  # breaks the ordering rule
    assert core.equihash_verify(p, inp, bad) == (False, "order")
    bad = s[:]
    bad[5] ^= 1
    assert core.equihash_verify(p, inp, bad)[0] is False
    assert core.equihash_verify(p, inp, s[:256]) == (False, "bad-size")
    dup = s[:256] + s[:256]
    assert core.equihash_verify(p, inp, dup)[0] is False


def test_small_params_exhaustive(core):
    """Equihash(48,5) (toy size) — solver and verifier agree on many nonces."""
    p = core.EquihashParams(48, 5)
    found = 0
    for nonce in range(6):
        inp = b"toy" + bytes([nonce]) * 29
        sols, _ = core.equihash_solve_cpu(p, inp, 16, 2)
        for s in sols:
            assert core.equihash_verify(p, inp, s) == (True, "")
        found += len(sols)
    assert found > 0
