"""GPU batch verification (program-as-data kernel) and the node's GPU miner."""
import random

import pytest

from kawpow_vectors import VECTORS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["dag", "dag-slab", "light"])
def test_verify_batch_multi_period_vs_cpu(core, gpu, mode):
    from nodexa_chain_core_amd.ops.verify import gpu_full_hash

    rng = random.Random(5)
    blocks = [rng.randrange(0, 7500) for _ in range(150)] + [7, 8, 9]  # many periods, epoch 0
    headers = [rng.randbytes(32) for _ in blocks]
    nonces = [rng.getrandbits(64) for _ in blocks]
    res = gpu_full_hash(blocks, headers, nonces, device=0, mode=mode)
    ctx = core.get_epoch_context(0)
    for i in range(0, len(blocks), 7):
        assert res[i] == core.kawpow_hash(ctx, blocks[i], headers[i], nonces[i]), i


@pytest.mark.parametrize("mode", ["dag", "dag-slab", "light"])
def test_verify_batch_reference_vectors(core, gpu, mode):
    from nodexa_chain_core_amd.ops.verify import gpu_full_hash

    vecs = [v for v in VECTORS if v[0] < 7500]
    res = gpu_full_hash([v[0] for v in vecs], [bytes.fromhex(v[1]) for v in vecs], [int(v[2], 16) for v in vecs],
                        device=0, mode=mode)
    for (block, _, _, mix, final), (f, m) in zip(vecs, res):
        assert (m.hex(), f.hex()) == (mix, final), block


def test_verify_light_other_epoch_and_mixed_batch(core, gpu):
    """Light mode at epoch 4 (reference vector) in one call with epoch-0 jobs."""
    from kawpow_vectors import HASH_30000

    from nodexa_chain_core_amd.ops.verify import gpu_full_hash

    block, header, nonce, mix, final = HASH_30000
    rng = random.Random(9)
    blocks = [block] + [rng.randrange(0, 7500) for _ in range(20)] + [block + 5]
    headers = [bytes.fromhex(header)] + [rng.randbytes(32) for _ in range(21)]
    nonces = [nonce] + [rng.getrandbits(64) for _ in range(21)]
    res = gpu_full_hash(blocks, headers, nonces, device=0, mode="light")
    assert (res[0][1].hex(), res[0][0].hex()) == (mix, final)
    ctx0, ctx4 = core.get_epoch_context(0), core.get_epoch_context(4)
    for i in (1, 10, 20):
        assert res[i] == core.kawpow_hash(ctx0, blocks[i], headers[i], nonces[i])
    assert res[-1] == core.kawpow_hash(ctx4, blocks[-1], headers[-1], nonces[-1])


def test_verify_light_batch_over_five_epochs(core, gpu):
    """One light batch over epochs 0-4: more epoch groups than the in-flight limit
    (ops/verify.MAX_RESIDENT_DAGS), so the groups run in two waves on the side streams; every row
    matches the host golden model."""
    from nodexa_chain_core_amd.ops.verify import MAX_RESIDENT_DAGS, gpu_full_hash

    rng = random.Random(11)
    blocks = [e * 7500 + rng.randrange(0, 7500) for e in range(5) for _ in range(6)]
    rng.shuffle(blocks)
    assert len({b // 7500 for b in blocks}) > MAX_RESIDENT_DAGS
    headers = [rng.randbytes(32) for _ in blocks]
    nonces = [rng.getrandbits(64) for _ in blocks]
    res = gpu_full_hash(blocks, headers, nonces, device=0, mode="light")
    for i, b in enumerate(blocks):
        assert res[i] == core.kawpow_hash(core.get_epoch_context(b // 7500), b, headers[i], nonces[i]), i


def test_node_gpu_mining_and_batch_verify(core, gpu, tmp_path):
    from nodexa_chain_core_amd.models.verify import verify_headers
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.rpc.client import RPCClient
    from nodexa_chain_core_amd.utils.config import ArgsManager

    addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
    args = ArgsManager()
    args.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                           f"-miningaddress={addr}", "-printtoconsole=0", "-gpus=0", "-gpuintensity=65536"])
    node = Node(args)
    node.start()
    try:
        c = RPCClient("127.0.0.1", node.rpc.port, "u", "p")
        hashes = c.generatetoaddress(5, addr)
        assert c.getblockcount() == 5
        info = c.getgpuinfo()
        assert info and info[0]["device"] == 0 and 0 in info[0]["epochs_resident"]
        hdrs = [node.state.chain.at_height(h).header for h in range(1, 6)]
        gpu_res = verify_headers(node.params, hdrs, gpus=[0])
        cpu_res = verify_headers(node.params, hdrs, gpus=None)
        assert all(r["valid"] for r in gpu_res) and gpu_res == cpu_res
        assert [r["hash"] for r in gpu_res] == hashes
        bad = core.BlockHeader.deserialize(hdrs[0].serialize(node.params.kawpow_activation_time),
                                           node.params.kawpow_activation_time)
        bad.nonce64 ^= 1
        r = verify_headers(node.params, [bad], gpus=[0])[0]
        assert not r["valid"]
    finally:
        node.stop()


def test_synthetic_chain_gpu_mixed(core, gpu):
    """GPU-mined synthetic chain (KawPow then Equihash era) is accepted by a fresh
    HeaderChain with full PoW checks, and the DAG scanner agrees with the CPU golden."""
    from nodexa_chain_core_amd.models import synthetic

    params, headers = synthetic.build_chain(40, 8, backend="gpu", seed=7)
    chain = core.HeaderChain(params)
    for h in headers:
        r = chain.accept_header(h, h.time + 7200, True)
        assert r.ok, r.reject
    assert sum(1 for h in headers if h.is_equihash()) == 8


def test_distributed_verify_single_rank_gpu():
    """parallel/verify.py on the GPU with one rank: same rows as the single-process path."""
    import os

    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import verify_headers
    from nodexa_chain_core_amd.parallel import world as W
    from nodexa_chain_core_amd.parallel.verify import verify_headers_distributed

    params, headers = synthetic.load(os.path.join(os.path.dirname(__file__), "data", "testnet_mixed_10k.hdr"))
    batch = headers[:300] + headers[-50:]
    W.init()
    try:
        got = verify_headers_distributed(params, batch, mode="light")
    finally:
        W.shutdown()
    assert got == verify_headers(params, batch, gpus=[0], mode="light")
    assert all(r["valid"] for r in got)


@pytest.mark.parametrize("fixture", ["testnet_kawpow_10k.hdr", "testnet_mixed_10k.hdr"])
def test_gpu_dgw_matches_host(core, gpu, fixture):
    """hip/kernels/dgw.hip against the host's DarkGravityWave: every DGW header of the 10k
    fixtures (bootstrap, KawPow switch, Equihash switch and overflow eras) gets exactly the nBits
    the host rules gave it; a tampered nBits is caught as bad-diffbits; process_headers takes
    the GPU path for the batch."""
    import os
    import struct

    import numpy as np

    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import process_headers
    from nodexa_chain_core_amd.ops import dgw

    params, headers = synthetic.load(os.path.join(os.path.dirname(__file__), "data", fixture))
    hs = list(headers)
    adj = headers[-1].time + 3600
    ref = core.HeaderChain(params)
    assert all(r.ok for r in ref.accept_headers(hs, adj, False))
    hashes = b"".join(ref.block_hash(h) for h in hs)
    times, bits, a, base = core.HeaderChain(params).dgw_series(hs, hashes)
    got = dgw.expected_bits(params, times, bits, a, len(hs), base, device=0)
    have = got != 0
    assert have.sum() >= len(hs) - 1  # every header with a parent in the DGW era
    want = np.array([h.bits for h in hs], dtype=np.uint32)
    assert np.array_equal(got[have], want[have])
    # accept with the GPU's nBits: same chain; a tampered header is refused at its index
    c = core.HeaderChain(params)
    assert all(r.ok for r in c.accept_headers(hs, adj, False, hashes, got.tobytes())) and c.tip().hash == ref.tip().hash
    bad = bytearray(got.tobytes())
    struct.pack_into("<I", bad, 4 * 5000, int(got[5000]) ^ 1)
    rc = core.HeaderChain(params).accept_headers(hs, adj, False, hashes, bytes(bad))
    assert len(rc) == 5001 and rc[-1].reject == "bad-diffbits"
    r = process_headers(core.HeaderChain(params), headers, adj, gpus=[0])
    assert r["accepted"] == len(hs) and r["dgw_gpu"]
