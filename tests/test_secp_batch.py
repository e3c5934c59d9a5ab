"""Batch ECDSA verification: the gfx950 kernel's arithmetic run on the host (CPU tier) and the
kernel itself (GPU tier) against the golden model (csrc/crypto/secp256k1.cpp), on valid
signatures, wrong messages, high-S forms, foreign keys, malformed DER and invalid keys."""
import random

import pytest

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def _der(r: int, s: int) -> bytes:
    def enc(x):
        b = x.to_bytes(32, "big").lstrip(b"\x00") or b"\x00"
        if b[0] & 0x80:
            b = b"\x00" + b
        return b"\x02" + bytes([len(b)]) + b
    body = enc(r) + enc(s)
    return b"\x30" + bytes([len(body)]) + body


def cases(core, n, seed=11):
    """(pub, sig, msg, expected) tuples, mixed valid and invalid."""
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        k = rng.randbytes(32)
        if not core.secp_seckey_valid(k):
            continue
        m = rng.randbytes(32)
        pub = core.secp_pubkey_create(k, rng.random() < 0.7)
        sig = core.secp_sign(m, k)
        kind = len(out) % 6
        if kind == 1:
            m = rng.randbytes(32)  # wrong message
        elif kind == 2:  # high-S form of a valid signature: accepted (normalised) like CPubKey::Verify
            rs = core.secp_der_to_rs(sig)
            r, s = int.from_bytes(rs[:32], "big"), int.from_bytes(rs[32:], "big")
            sig = _der(r, N - s)
        elif kind == 3:
            pub = core.secp_pubkey_create(rng.randbytes(31) + b"\x01")  # someone else's key
        elif kind == 4:
            sig = sig[:-1]  # truncated DER
        elif kind == 5 and len(out) % 12 == 5:
            pub = b"\x02" + b"\xff" * 32  # x >= p: not a key
        out.append((pub, sig, m, bool(core.secp_verify(pub, sig, m))))
    return out


def test_model32_matches_golden(core):
    cs = cases(core, 48)
    assert any(e for *_, e in cs) and not all(e for *_, e in cs)
    for pub, sig, m, expect in cs:
        v = core.secp_verify_model32(pub, sig, m)
        assert v in (0, 1, 2)
        if v != 2:
            assert (v == 1) == expect, (pub.hex(), sig.hex(), m.hex())


def test_pack_jobs_layout(core):
    cs = cases(core, 4)
    packed = core.secp_pack_jobs([(p, s, m) for p, s, m, _ in cs])
    assert len(packed) == 4 * core.SECP_JOB_BYTES == 4 * 176


@pytest.mark.gpu
def test_gpu_batch_verify_matches_golden(core, gpu):
    from nodexa_chain_core_amd.ops import secp

    cs = cases(core, 1000, seed=5)
    got = secp.verify_batch([(p, s, m) for p, s, m, _ in cs], device=0)
    assert got == [e for *_, e in cs]
