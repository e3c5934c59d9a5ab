"""X16R / X16RV2 primitives and chaining vs golden digests.

tests/data/x16r_vectors.json is produced by tools/ref_x16r_vectors.sh, which
compiles the reference's own sph sources (src/algo/*.c, src/algo/tiger.cpp) on
the host and hashes deterministic inputs of 0..1000 bytes; `chains` are whole
X16R / X16RV2 hashes of random 80-byte headers whose hashPrevBlock forces every
algorithm into every slot (src/hash.h:320-327,335-605).
"""
import json
import os

import pytest

from nodexa_chain_core_amd import core

_core = core()
VEC = json.load(open(os.path.join(os.path.dirname(__file__), "data", "x16r_vectors.json")))
NAMES = ["blake512", "bmw512", "groestl512", "jh512", "keccak512", "skein512", "luffa512", "cubehash512",
         "shavite512", "simd512", "echo512", "hamsi512", "fugue512", "shabal512", "whirlpool", "sha512", "tiger"]


@pytest.mark.parametrize("slot", range(17), ids=NAMES)
def test_primitive(slot):
    for inp, out in VEC["primitives"][NAMES[slot]]:
        got = _core.x16r_algo(slot, bytes.fromhex(inp))
        n = len(out) // 2
        assert got[:n].hex() == out, (NAMES[slot], len(inp) // 2)
        if slot == 16:
            assert got[n:] == bytes(64 - n)  # tiger is zero-extended to 64 bytes (uint512 ctor)


def test_every_slot_available():
    assert all(_core.x16r_slot_available(a) for a in range(16))


@pytest.mark.parametrize("v2", [False, True], ids=["x16r", "x16rv2"])
def test_chains(v2):
    for c in VEC["chains"]:
        hdr, prev = bytes.fromhex(c["header"]), bytes.fromhex(c["prev"])
        got = (_core.x16rv2 if v2 else _core.x16r)(hdr, prev)
        assert got.hex() == c["x16rv2" if v2 else "x16r"]


def test_x16r_groups_matches_selections():
    """_core.x16r_groups (the GPU batch's launch tables) is a stable grouping of every step's
    headers by the selection nibble ops/x16r.selections reads."""
    import numpy as np

    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.ops.x16r import selections

    rng = np.random.default_rng(4)
    for n in (1, 7, 1000):
        hdr = rng.integers(0, 256, size=(n, 80), dtype=np.uint8)
        order_b, offsets = _core.x16r_groups(hdr)
        order = np.frombuffer(order_b, dtype=np.int32).reshape(16, n)
        offsets = np.asarray(offsets).reshape(16, 17)
        sel = selections(hdr)
        for s in range(16):
            assert (order[s] == np.argsort(sel[:, s], kind="stable")).all()
            assert (offsets[s, 1:] == np.cumsum(np.bincount(sel[:, s], minlength=16))).all()
            assert offsets[s, 0] == 0
    with pytest.raises(ValueError):
        _core.x16r_groups(b"\0" * 79)
