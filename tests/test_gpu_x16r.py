"""gfx950 X16R / X16RV2 batch hashing (hip/kernels/x16r.hip) vs the reference-derived chain
vectors and the host implementation."""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VEC = json.load(open(os.path.join(os.path.dirname(__file__), "data", "x16r_vectors.json")))


def test_reference_chain_vectors(core, gpu):
    from nodexa_chain_core_amd.ops.x16r import x16r_hash_batch

    hdrs = b"".join(bytes.fromhex(c["header"]) for c in VEC["chains"])
    for v2, key in ((False, "x16r"), (True, "x16rv2")):
        got = x16r_hash_batch(hdrs, v2=v2)
        assert [bytes(r).hex() for r in got] == [c[key] for c in VEC["chains"]]


def test_random_batch_mixed_versions_vs_host(core, gpu):
    from nodexa_chain_core_amd.ops.x16r import x16r_hash_batch

    rng = random.Random(3)
    n = 1500
    hdrs = [rng.randbytes(80) for _ in range(n)]
    v2 = np.array([rng.random() < 0.5 for _ in range(n)])
    got = x16r_hash_batch(b"".join(hdrs), v2=v2)
    for i in range(0, n, 7):  # the host chain is the slow side
        fn = core.x16rv2 if v2[i] else core.x16r
        assert bytes(got[i]) == fn(hdrs[i], hdrs[i][4:36]), i


def test_verify_headers_legacy_batch_on_gpu_matches_host(core, gpu):
    """models/verify routes a legacy (pre-KawPow) batch of X16R_GPU_MIN headers or more through the
    GPU hash: same verdicts and hashes as the host cores, X16R and X16RV2 by nTime."""
    from nodexa_chain_core_amd.chain.state import REGTEST_KAWPOW_FROM_GENESIS, make_params
    from nodexa_chain_core_amd.models import verify as MV

    params = make_params("regtest", REGTEST_KAWPOW_FROM_GENESIS)
    # KawPow-regtest activates KawPow before X16RV2: move X16RV2 inside the legacy era for this batch
    params.x16rv2_activation_time = params.kawpow_activation_time - 100_000
    rng = random.Random(5)
    hs = []
    for i in range(MV.X16R_GPU_MIN + 40):
        h = core.BlockHeader()
        h.version = 0x20000000
        h.prev = rng.randbytes(32)
        h.merkle_root = rng.randbytes(32)
        h.time = params.x16rv2_activation_time + rng.choice([-1000, 1000])  # both versions
        h.bits = 0x207fffff  # regtest limit: about half of the hashes meet it
        h.nonce = rng.getrandbits(32)
        hs.append(h)
    assert all(h.time < params.kawpow_activation_time for h in hs)
    gpu_r = MV.verify_headers(params, hs, gpus=[0])
    cpu_r = MV.verify_headers(params, hs, gpus=None)
    assert [(r["valid"], r["hash"]) for r in gpu_r] == [(r["valid"], r["hash"]) for r in cpu_r]
    assert 0 < sum(r["valid"] for r in gpu_r) < len(hs)


def test_gpu_search_matches_host_search(core, gpu):
    """X16rSearcher finds the same lowest nonce (and hash) as the host's x16r_search, over windows
    that end with and without a hit, X16R and X16RV2."""
    from nodexa_chain_core_amd.ops.x16r import X16rSearcher

    s = X16rSearcher(0, window=4096)
    rng = random.Random(8)
    for v2 in (False, True):
        hdr = rng.randbytes(80)
        target = (1 << 248).to_bytes(32, "little")  # ~1 in 256 hashes
        got, hashes = s.search(hdr, v2, target, 1000, 20000)
        want, _ = core.x16r_search(hdr, v2, target, 1000, 20000)
        assert got is not None and want is not None
        assert (got[0], got[1]) == (int(want[0]), bytes(want[1]))
        assert hashes == got[0] - 1000 + 1
        none, n = s.search(hdr, v2, bytes(32), 0, 5000)  # nothing meets a zero target
        assert none is None and n == 5000


def test_node_miner_legacy_blocks_on_gpu(core, gpu):
    """The mining loop's X16R / X16RV2 windows run on the GPU (LegacyGpuDevice) and find blocks
    the host accepts."""
    from nodexa_chain_core_amd.miner.search import ALGO_X16R, LegacyGpuDevice, Work

    dev = LegacyGpuDevice(0, window=1 << 14)
    hdr = bytearray(random.Random(2).randbytes(80))
    boundary = ((1 << 256) // 64).to_bytes(32, "big")  # ~1 in 64
    w = Work(header=bytes(hdr), boundary=boundary, height=5, algo=ALGO_X16R)
    dev.submit(0, w, 0, 1 << 14)
    r = dev.wait(0)
    assert r.shares, r
    sh = r.shares[0]
    h = bytearray(hdr)
    h[76:80] = sh.nonce.to_bytes(4, "little")
    assert core.x16r(bytes(h), bytes(h[4:36])) == sh.block_hash
    assert int.from_bytes(sh.block_hash, "little") <= int.from_bytes(boundary, "big")
