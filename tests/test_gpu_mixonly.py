"""SURVEY K4 + K6 on the MI355X: the fused SHA256d + mix-only KawPow check (progpow::hash_no_verify,
src/crypto/ethash/lib/ethash/progpow.cpp:498-550) gives, for every header of the committed 10k
fixture and of mutated copies (wrong mix, unusual / negative / overflowing nBits), exactly the job
records, boundaries and prefilter verdicts of the native host pass."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(__file__), "data", "testnet_mixed_10k.hdr")


def test_gpu_prefilter_matches_host_pass(core, gpu):
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import _prepare_gpu

    params, headers = synthetic.load(FIXTURE)
    act = params.kawpow_activation_time
    rng = random.Random(3)
    extra = []
    for bits in (0x1d00ffff, 0x207fffff, 0x03123456, 0x01003456, 0x04923456, 0x23000001, 0x2200ffff, 0x20800000):
        h = core.BlockHeader.deserialize(headers[rng.randrange(len(headers))].serialize(act), act)
        if h.is_equihash():
            continue
        h.bits = bits
        extra.append(h)
    for _ in range(64):  # a flipped byte of the claimed mix: the prefilter must reject most of these
        h = core.BlockHeader.deserialize(headers[rng.randrange(len(headers))].serialize(act), act)
        if h.is_equihash():
            continue
        m = bytearray(h.mix_hash)
        m[rng.randrange(32)] ^= 0x40
        h.mix_hash = bytes(m)
        extra.append(h)
    batch = list(headers) + extra
    want = core.kawpow_batch_prepare(batch, act)
    got = _prepare_gpu(params, batch, 0)
    kinds_w, kinds_g = np.frombuffer(want[0], np.uint8), np.frombuffer(got[0], np.uint8)
    assert (kinds_w == kinds_g).all()
    kp = np.flatnonzero(kinds_w < 2)
    for k, width in ((1, 48), (2, 32), (3, 32), (4, 32)):
        w = np.frombuffer(want[k], np.uint8).reshape(-1, width)[kp]
        g = np.frombuffer(got[k], np.uint8).reshape(-1, width)[kp]
        assert (w == g).all(), k
    assert (kinds_w[len(headers):] == 1).sum() >= 40  # most mutated mixes fail the cheap check
