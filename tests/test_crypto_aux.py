"""Auxiliary hashes against public test vectors and Python's hashlib/hmac."""
import hashlib
import hmac
import os

import pytest

from nodexa_chain_core_amd import core

_core = core()


@pytest.mark.parametrize("n", [0, 1, 3, 55, 56, 63, 64, 65, 119, 128, 1000])
def test_sha1_sha512_ripemd_vs_hashlib(n):
    d = os.urandom(n)
    assert _core.sha1(d) == hashlib.sha1(d).digest()
    assert _core.sha512(d) == hashlib.sha512(d).digest()
    try:
        ref = hashlib.new("ripemd160", d).digest()
    except ValueError:  # OpenSSL without legacy provider
        ref = None
    if ref is not None:
        assert _core.ripemd160(d) == ref


def test_ripemd160_vectors():
    assert _core.ripemd160(b"").hex() == "9c1185a5c5e9fc54612808977ee8f548b2258d31"
    assert _core.ripemd160(b"abc").hex() == "8eb208f7e05d987a9b044a8e98c6b087f15a0bfc"


@pytest.mark.parametrize("klen", [0, 20, 64, 65, 131])
def test_hmac(klen):
    k, d = os.urandom(klen), os.urandom(77)
    assert _core.hmac_sha256(k, d) == hmac.new(k, d, hashlib.sha256).digest()
    assert _core.hmac_sha512(k, d) == hmac.new(k, d, hashlib.sha512).digest()


def test_siphash_reference_vector_and_uint256():
    k0 = int.from_bytes(bytes(range(8)), "little")
    k1 = int.from_bytes(bytes(range(8, 16)), "little")
    # Aumasson & Bernstein, SipHash paper appendix: 15-byte message 00..0e
    assert _core.siphash24(k0, k1, bytes(range(15))) == 0xa129ca6149be45e5
    v = os.urandom(32)
    assert _core.siphash_uint256(k0, k1, v) == _core.siphash24(k0, k1, v)
    assert _core.siphash_uint256_extra(k0, k1, v, 0x1234) == _core.siphash24(k0, k1, v + (0x1234).to_bytes(4, "little"))


def test_murmur3_vectors():
    # Appleby's MurmurHash3_x86_32 (also BIP37 bloom-filter test values)
    assert _core.murmur3_32(0, b"") == 0
    assert _core.murmur3_32(1, b"") == 0x514E28B7
    assert _core.murmur3_32(0xffffffff, b"") == 0x81F16F39
    assert _core.murmur3_32(0, b"\x00\x00\x00\x00") == 0x2362F9DE
    assert _core.murmur3_32(0x9747b28c, b"Hello, world!") == 0x24884CBA


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 127, 128, 129, 1000, 65537])
def test_sha256_paths_vs_hashlib(n):
    d = os.urandom(n)
    assert _core.sha256(d) == hashlib.sha256(d).digest()
    assert _core.sha256d(d) == hashlib.sha256(hashlib.sha256(d).digest()).digest()
