"""CPU golden KawPow / ethash model vs the reference's fixtures
(src/test/kawpow_tests.cpp:20-140, src/crypto/ethash/progpow_test_vectors.hpp)."""
import pytest

from kawpow_vectors import EMPTY_1000, HASH_30000, L1_EPOCH0_FIRST20, VECTORS


def test_epoch_sizes(core):
    # spec values: epoch 0 light cache 262139 items, dataset 8388593 items (1024-bit)
    assert core.light_cache_num_items(0) == 262139
    assert core.full_dataset_num_items(0) == 8388593
    assert core.find_largest_prime(10) == 7
    assert core.find_largest_prime(2) == 2
    # epoch seed chain and inverse
    assert core.epoch_seed(0) == bytes(32)
    assert core.epoch_seed(1) == core.keccak256(bytes(32))
    assert core.find_epoch_number(core.epoch_seed(17)) == 17


def test_keccak_known_answers(core):
    # original Keccak-256 / 512 of the empty string
    assert core.keccak256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert core.keccak512(b"").hex().startswith("0eab42de4c3ceb9235fc91acffe746b29c29a8c366b7c60e4e67c466f36a4304")
    assert core.sha256(b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"


def test_l1_cache(ctx0):
    assert ctx0.l1[:20] == L1_EPOCH0_FIRST20


def test_hash_empty(core, ctx0):
    f, m = core.kawpow_hash(ctx0, 1, bytes(32), 0)
    assert (m.hex(), f.hex()) == EMPTY_1000


def test_vectors_hash_and_verify(core):
    ctx = None
    for block, header, nonce, mix, final in VECTORS:
        epoch = block // 7500
        if ctx is None or ctx.epoch != epoch:
            ctx = core.get_epoch_context(epoch)
        h = bytes.fromhex(header)
        n = int(nonce, 16)
        f, m = core.kawpow_hash(ctx, block, h, n)
        assert m.hex() == mix and f.hex() == final, block
        assert core.kawpow_verify(ctx, block, h, m, n, f)
        lower = bytearray(f)
        lower[31] = (lower[31] - 1) & 0xFF
        assert not core.kawpow_verify(ctx, block, h, m, n, bytes(lower))
        bad_mix = bytearray(m)
        bad_mix[7] = (bad_mix[7] + 1) & 0xFF
        assert not core.kawpow_verify(ctx, block, h, bytes(bad_mix), n, f)
        assert core.kawpow_hash_no_verify(block, h, m, n) == f


def test_hash_30000(core):
    block, header, nonce, mix, final = HASH_30000
    ctx = core.get_epoch_context(block // 7500)
    f, m = core.kawpow_hash(ctx, block, bytes.fromhex(header), nonce)
    assert (m.hex(), f.hex()) == (mix, final)


def test_search_light_and_full(core, ctx0):
    boundary = bytes.fromhex("00" + "ff" * 31)
    ok, nonce, f, m = core.kawpow_search_light(ctx0, 0, bytes(32), boundary, 700, 100)
    assert not ok
    ok, nonce, f, m = core.kawpow_search_light(ctx0, 0, bytes(32), boundary, 300, 100)
    assert ok and nonce == 395
    dag = core.HostDag(ctx0)  # lazily filled host DAG
    ok2, nonce2, f2, m2 = core.kawpow_search_full(dag, 0, bytes(32), boundary, 300, 100, 4)
    assert ok2 and nonce2 == 395 and f2 == f and m2 == m
    assert core.kawpow_hash(ctx0, 0, bytes(32), 395) == (f, m)


def test_program_shape(core):
    p = core.make_kawpow_program(0)
    cache, math, dag = p.cache_ops(), p.math_ops(), p.dag_ops()
    assert len(cache) == 11 and len(math) == 18 and len(dag) == 4
    assert dag[0][0] == 0
    for src1, src2, _, dst, _ in math:
        assert src1 != src2 and 0 <= dst < 32
    src = core.kawpow_codegen_hip(0)
    assert "KAWPOW_PROGRAM" in src and "KAWPOW_DAG_MERGE" in src


def test_dataset_items_consistent(core, ctx0):
    item = core.dataset_item_2048(ctx0, 5)
    assert item[:64] == core.dataset_item_512(ctx0, 20)
    assert item[192:] == core.dataset_item_512(ctx0, 23)


def test_ethash_classic_roundtrip(core, ctx0):
    f, m = core.ethash_hash(ctx0, bytes(32), 7)
    assert core.ethash_verify(ctx0, bytes(32), m, 7, f)
    assert not core.ethash_verify(ctx0, bytes(32), bytes(32), 7, f)


def test_light_cache_disk_cache(core, tmp_path):
    """-dagcache: a light cache written to disk reloads bit-identically; a corrupted file
    is detected by its checksum and rebuilt (SURVEY §5 checkpoint/resume)."""
    import glob

    core.set_light_cache_dir(str(tmp_path))
    try:
        a = core.create_epoch_context(1)
        files = glob.glob(str(tmp_path / "light-1-*.bin"))
        assert len(files) == 1
        b = core.create_epoch_context(1)  # loaded from disk
        assert a.light_cache() == b.light_cache() and a.l1 == b.l1
        with open(files[0], "r+b") as f:
            f.seek(100)
            f.write(b"\xff\xff")
        c = core.create_epoch_context(1)  # checksum mismatch -> rebuilt
        assert c.light_cache() == a.light_cache()
    finally:
        core.set_light_cache_dir("")


def test_search_variant_selection_by_dag_size(core):
    """ops/jit.defines_for: the 32-bit buffer-offset DAG loads (KP_SBUFFER) are used below 4 GiB
    only (epoch 384 is 4294962304 bytes; epoch 385 is above 2^32); above, the 64-bit form
    (KP_PTR64) keeps the 768-thread / 6-wave tuning."""
    from nodexa_chain_core_amd.ops import jit

    below = core.full_dataset_num_items(384) * 128
    above = core.full_dataset_num_items(385) * 128
    assert below < 1 << 32 <= above
    small = jit.defines_for(below, jit.TUNED_DEFINES)
    big = jit.defines_for(above, jit.TUNED_DEFINES)
    assert "KP_SBUFFER" in small and "KP_PTR64" not in small
    assert "KP_SBUFFER" not in big and "KP_PTR64" in big and "KP_DPP" in big
    for d in (small, big):
        assert {"KP_BLOCK=768", "KP_MIN_WAVES=6", "KP_SCHED_FENCE", "KP_NT_DAG"} <= set(d)
    assert jit.defines_for(above, ("KP_SBUFFER", "KP_DPP")) == ("KP_PTR64", "KP_DPP")




def test_prefetch_contexts_builds_in_parallel(core):
    """ops/verify.prefetch_contexts: the light caches of a batch's new epochs are built side by
    side (the native build releases the GIL) and land in the native LRU the verify paths read."""
    import time

    from nodexa_chain_core_amd.ops import verify as V

    V.prefetch_contexts([7, 8], device=0)
    t = time.perf_counter()
    a, b = core.get_epoch_context(7), core.get_epoch_context(8)
    assert time.perf_counter() - t < 0.2  # LRU hits, not two ~1 s builds
    assert a.light_items > 0 and b.light_items > a.light_items
