"""gfx950 DAG build + KawPow search/hash vs the CPU golden model and the
reference's fixtures. Every test here runs the native HIP path (no fallback)."""
import os
import random

import pytest

from kawpow_vectors import VECTORS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def epoch0(gpu, core):
    from nodexa_chain_core_amd.ops.ethash import DeviceEpoch

    e = DeviceEpoch(0, device=0, ctx=core.get_epoch_context(0))
    e.build()
    import torch

    torch.cuda.synchronize()
    return e


def test_dag_l1_and_items(core, epoch0):
    assert epoch0.l1_matches()
    rng = random.Random(7)
    idx = [0, 1, 255, 256, epoch0.items512 - 1] + [rng.randrange(epoch0.items512) for _ in range(24)]
    for i in idx:
        assert epoch0.item512(i) == core.dataset_item_512(epoch0.ctx, i), i


def test_search_matches_reference_search(core, epoch0):
    from nodexa_chain_core_amd.ops.kawpow import KawpowSearcher

    s = KawpowSearcher(epoch0, 0)
    boundary = bytes.fromhex("00" + "ff" * 31)
    shares = s.search(bytes(32), 300, 256, boundary)
    assert shares and shares[0].nonce == 395  # reference kawpow_tests.cpp: first solution is 395
    f, m = core.kawpow_hash(epoch0.ctx, 0, bytes(32), 395)
    assert shares[0].final_hash == f and shares[0].mix_hash == m
    for sh in shares:
        assert sh.verify_host(0, bytes(32), boundary)
        assert core.kawpow_verify(epoch0.ctx, 0, bytes(32), sh.mix_hash, sh.nonce, boundary)
    assert not [x for x in s.search(bytes(32), 512, 512, boundary) if 700 <= x.nonce < 800]


def test_hash_batch_vectors_epoch0(core, epoch0):
    from nodexa_chain_core_amd.ops.kawpow import KawpowSearcher

    for block, header, nonce, mix, final in VECTORS:
        if block // 7500 != 0:
            continue
        s = KawpowSearcher(epoch0, block)
        (f, m), = s.hash_batch([bytes.fromhex(header)], [int(nonce, 16)])
        assert m.hex() == mix and f.hex() == final, block


def test_hash_batch_random_vs_cpu(core, epoch0):
    from nodexa_chain_core_amd.ops.kawpow import KawpowSearcher

    rng = random.Random(11)
    s = KawpowSearcher(epoch0, 4242)
    headers = [rng.randbytes(32) for _ in range(300)]
    nonces = [rng.getrandbits(64) for _ in range(300)]
    out = s.hash_batch(headers, nonces)
    for i in range(0, 300, 37):
        assert out[i] == core.kawpow_hash(epoch0.ctx, 4242, headers[i], nonces[i])


@pytest.mark.skipif(os.environ.get("NODEXA_FAST_GPU_TESTS") == "1", reason="multi-epoch DAG builds")
def test_vectors_other_epochs(core, gpu):
    import torch

    from nodexa_chain_core_amd.ops.ethash import DeviceEpoch
    from nodexa_chain_core_amd.ops.kawpow import KawpowSearcher

    by_epoch = {}
    for v in VECTORS:
        by_epoch.setdefault(v[0] // 7500, []).append(v)
    for epoch, vecs in sorted(by_epoch.items()):
        if epoch == 0:
            continue
        e = DeviceEpoch(epoch, device=0, ctx=core.get_epoch_context(epoch))
        e.build()
        torch.cuda.synchronize()
        assert e.l1_matches()
        for block, header, nonce, mix, final in vecs:
            s = KawpowSearcher(e, block)
            (f, m), = s.hash_batch([bytes.fromhex(header)], [int(nonce, 16)])
            assert (m.hex(), f.hex()) == (mix, final), block
        del e
        torch.cuda.empty_cache()


def test_next_epoch_dag_prebuild(core, gpu):
    """Within PREBUILD_WINDOW blocks of an epoch boundary the backend builds the next
    epoch's DAG on a side stream; the first block of the new epoch then finds it resident
    and a search there is bit-exact against the golden model."""
    from nodexa_chain_core_amd.miner.kawpow_miner import GpuKawpowBackend

    be = GpuKawpowBackend(0, intensity=1 << 16)
    last = core.EPOCH_LENGTH - 5  # block 7495, epoch 0
    t = be.maybe_prebuild(last)
    assert t is not None
    t.join(120)
    assert 1 in be.epochs and be.prebuilt_epochs == [1]
    assert be.maybe_prebuild(last) is None  # already resident
    hh = core.sha256d(b"prebuild")
    res = be.search(core.EPOCH_LENGTH, hh, bytes.fromhex("0f" + "ff" * 31), 0, 1 << 12)
    assert res is not None
    nonce, mix, fin = res
    ctx = core.get_epoch_context(1)
    assert core.kawpow_hash(ctx, core.EPOCH_LENGTH, hh, nonce) == (fin, mix)
