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
def test_classic_hashimoto_batch_vs_cpu(core, epoch0):
    """ethash_hashimoto.hip (classic Ethash over the resident DAG) against the host's ethash_hash
    for random header hashes and nonces, plus a batch size that leaves a partial last block."""
    rng = random.Random(11)
    n = 37
    hh = [rng.randbytes(32) for _ in range(n)]
    nonces = [rng.getrandbits(64) for _ in range(n)]
    nonces[0], hh[0] = 7, bytes(32)
    got = epoch0.hashimoto_batch(hh, nonces)
    for h, nonce, (f, m) in zip(hh, nonces, got):
        assert (f, m) == core.ethash_hash(epoch0.ctx, h, nonce), nonce
        assert core.ethash_verify(epoch0.ctx, h, m, nonce, f)


def test_classic_ethash_search_vs_cpu(core, epoch0):
    """ethash_search (device-side nonces and boundary check) returns the first nonce the host's
    sequential ethash_hash loop finds, with its final and mix hashes; a boundary nothing meets in
    the range returns None."""
    hh = bytes(range(32))
    boundary = bytes.fromhex("0f" + "ff" * 31)
    got = epoch0.ethash_search(hh, boundary, 1000, 200, window=64)  # several windows
    nonce = next(n for n in range(1000, 1200) if core.ethash_hash(epoch0.ctx, hh, n)[0] <= boundary)
    f, m = core.ethash_hash(epoch0.ctx, hh, nonce)
    assert got == (nonce, f, m)
    assert epoch0.ethash_search(hh, bytes(32), 0, 300) is None


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
    """The mining service prebuilds the next epoch's DAG on a side stream (GpuSearchDevice.prebuild,
    voted in by every rank near the boundary); the first block of the new epoch then finds it
    resident, and a search there is bit-exact against the golden model."""
    import torch

    from nodexa_chain_core_amd.miner.search import GpuSearchDevice, SearchPipeline, Work

    dev = GpuSearchDevice(0)
    dev.searcher(core.EPOCH_LENGTH - 5)  # epoch 0 resident (block 7495)
    dev.prebuild(1)
    assert 1 in dev.pending_build and not dev.epoch_ready(1)
    dev.prebuild(1)  # idempotent
    hh = core.sha256d(b"prebuild")
    w = Work(hh, bytes.fromhex("0f" + "ff" * 31), core.EPOCH_LENGTH, 1, 0, 0)
    pipe = SearchPipeline(dev, watchdog_s=120)
    pipe.step(w, 0, 1 << 12)
    res = pipe.drain()
    assert dev.epoch_ready(1) and not dev.pending_build and res.shares
    ctx = core.get_epoch_context(1)
    for sh in res.shares[:4]:
        assert core.kawpow_hash(ctx, core.EPOCH_LENGTH, hh, sh.nonce) == (sh.final_hash, sh.mix_hash)
    dev.close()
    torch.cuda.empty_cache()


def _headline_epoch(core, epoch):
    import torch

    from nodexa_chain_core_amd.ops.ethash import DeviceEpoch

    e = DeviceEpoch(epoch, device=0, ctx=core.get_epoch_context(epoch))
    e.build()
    torch.cuda.synchronize()
    assert e.l1_matches()
    return e


@pytest.mark.parametrize("epoch", [384, 390])
def test_shipped_variant_full_hash_at_headline_epochs(core, gpu, epoch):
    """The kernel variant that ships at each DAG size — epoch 384 (4.00 GiB: structured-buffer
    loads, 768 threads, register digests, scheduling fences) and epoch 390 (4.05 GiB: the same form
    with 64-bit item addresses, KP_PTR64) — hashes bit-exactly like the host golden model (_core.kawpow_hash, light mode),
    both through hash_batch and through search (every share of a window re-hashed in full)."""
    import torch

    from nodexa_chain_core_amd.ops import jit
    from nodexa_chain_core_amd.ops.kawpow import KawpowSearcher

    e = _headline_epoch(core, epoch)
    height = epoch * core.EPOCH_LENGTH + 123
    s = KawpowSearcher(e, height)
    variant = jit.defines_for(e.dag_bytes)
    assert ("KP_SBUFFER" in variant) == (epoch == 384) and ("KP_PTR64" in variant) == (epoch == 390)
    assert "KP_BLOCK=768" in variant and s.block == 768
    rng = random.Random(epoch)
    headers = [rng.randbytes(32) for _ in range(64)]
    nonces = [rng.getrandbits(64) for _ in range(64)]
    out = s.hash_batch(headers, nonces)
    for i in range(0, 64, 9):
        assert out[i] == core.kawpow_hash(e.ctx, height, headers[i], nonces[i]), (epoch, i)
    hh = core.sha256d(b"headline-%d" % epoch)
    shares = s.search(hh, 1 << 40, s.block * 64, bytes.fromhex("07" + "ff" * 31))  # ~1/32 pass
    assert len(shares) >= 8
    for sh in shares[:12]:
        assert sh.verify_full(height, hh, ctx=e.ctx), (epoch, sh.nonce)
    del s, e
    torch.cuda.empty_cache()


def test_corrupted_dag_item_is_caught(core, gpu):
    """A damaged DAG row makes the full host re-hash reject the GPU's result (the mix-only check
    would accept it: the final hash is consistent with the GPU's own wrong mix)."""
    import torch

    from nodexa_chain_core_amd.ops.ethash import DeviceEpoch
    from nodexa_chain_core_amd.ops.kawpow import KawpowSearcher, Share

    e = DeviceEpoch(0, device=0, ctx=core.get_epoch_context(0))
    e.build()
    torch.cuda.synchronize()
    height, hh, nonce = 5, core.sha256d(b"corrupt"), 77
    s = KawpowSearcher(e, height)
    (f, m), = s.hash_batch([hh], [nonce])
    assert Share(nonce, m, f).verify_full(height, hh, ctx=e.ctx)
    rows = e.dag.view(torch.int32)
    rows = rows[:rows.numel() // 64 * 64].view(-1, 64)
    rows[64:, :] ^= 0x01000000  # every item this nonce can gather outside the L1
    torch.cuda.synchronize()
    (f2, m2), = s.hash_batch([hh], [nonce])
    bad = Share(nonce, m2, f2)
    assert (f2, m2) != (f, m)
    assert bad.verify_host(height, hh)          # mix-only: consistent with its own mix
    assert not bad.verify_full(height, hh, ctx=e.ctx)  # full re-hash: caught


def test_pipelined_search_loop_on_gpu(core, gpu):
    """miner/search: two windows in flight, ring copies behind each kernel, the generation word
    aborting a queued window, exact hash accounting, shares re-hashed in full."""
    import time

    from nodexa_chain_core_amd.miner.search import GpuSearchDevice, SearchPipeline, Work

    dev = GpuSearchDevice(0)
    height = 4242
    hh = core.sha256d(b"pipeline")
    w = Work(hh, bytes.fromhex("0001" + "ff" * 30), height, 1, 0, 0)  # ~1 in 32768 passes
    pipe = SearchPipeline(dev, watchdog_s=60)
    block = dev.block_for(height)
    n = block * 512
    assert pipe.step(w, 0, n) is None
    r0 = pipe.step(w, n, n)
    assert r0.hashes == n and r0.start == 0 and 2 <= len(r0.shares) < 64  # ~12 expected, ring not full
    ctx = core.get_epoch_context(0)
    for sh in r0.shares[:6]:
        assert sh.verify_full(height, hh, w.boundary, ctx=ctx)
    # a big window queued behind the running one, then the template changes: it stops early
    big = block * 40000
    pipe.step(w, 2 * n, big)
    dev.abort()
    t0 = time.time()
    r_big = pipe.drain()
    assert r_big.hashes < big // 4 and time.time() - t0 < 5
    dev.close()
