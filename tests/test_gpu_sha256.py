"""HIP batch SHA-256d (hip/kernels/sha256d.hip) against the host (hashlib / C++ core)."""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sha256d(b: bytes) -> bytes:
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()


@pytest.mark.parametrize("length", [0, 1, 55, 56, 63, 64, 80, 119, 120, 1459])
def test_sha256d_batch_lengths(length):
    from nodexa_chain_core_amd.ops.sha256 import sha256d_batch

    rng = np.random.default_rng(length)
    msgs = rng.integers(0, 256, (300, length), dtype=np.uint8)
    got = sha256d_batch(msgs)
    want = [_sha256d(m.tobytes()) for m in msgs]
    assert [g.tobytes() for g in got] == want


def test_merkle_root_matches_core(core):
    from nodexa_chain_core_amd.ops.sha256 import merkle_root

    for n in (1, 2, 3, 7, 8, 1000, 4097):
        txids = [os.urandom(32) for _ in range(n)]
        assert merkle_root(txids) == core.compute_merkle_root(txids)[0]


def test_header_hashes_match_core(core):
    """KawPow header hashes of the 10k fixture (GetKAWPOWHeaderHash) on the device."""
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.ops.sha256 import sha256d_batch

    params, headers = synthetic.load(os.path.join(os.path.dirname(__file__), "data", "testnet_kawpow_10k.hdr"))
    got = sha256d_batch([h.kawpow_input() for h in headers])
    assert all(g.tobytes() == h.kawpow_header_hash() for g, h in zip(got, headers))
