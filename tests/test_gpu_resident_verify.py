"""Device-resident batch header verify (ops/header_batch.py, models/verify.process_batch_resident;
BASELINE config 5): one upload, PoW + block hashes + DGW nBits on the GPU, one download, the serial
index insert on the host. Must give the same chain and the same first rejection (index and
reason) as the host path (HeaderChain.accept_headers with the CPU golden PoW)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DATA = os.path.join(os.path.dirname(__file__), "data")


def _load(core, fixture):
    from nodexa_chain_core_amd.models import synthetic

    params, headers = synthetic.load(os.path.join(DATA, fixture))
    raw = open(os.path.join(DATA, fixture), "rb").read()
    return params, list(headers), raw


def _chain(core, params, fixture):
    """A fresh chain for `fixture`: genesis, plus its stored-index anchor when it starts past genesis
    (the headline-epoch fixture, heights 2,880,000-2,889,999)."""
    from nodexa_chain_core_amd.models import synthetic

    return synthetic.new_chain(params, synthetic.load_anchor(os.path.join(DATA, fixture), params))


@pytest.mark.parametrize("fixture", ["testnet_kawpow_10k.hdr", "testnet_mixed_10k.hdr", "testnet_mixed_e384_10k.hdr"])
def test_resident_matches_host_chain(core, gpu, fixture):
    """Epochs 0-1 and the headline epochs 384-385 (4 GiB DAGs)."""
    from nodexa_chain_core_amd.models.verify import process_batch_resident

    params, hs, raw = _load(core, fixture)
    act = params.kawpow_activation_time
    adj = hs[-1].time + 3600
    ref = _chain(core, params, fixture)
    assert all(r.ok for r in ref.accept_headers(hs, adj, False))
    batch = core.HeaderBatch.from_bytes(raw, act)
    for _ in range(2):  # cold (epoch DAGs, program tables) and warm
        c = _chain(core, params, fixture)
        r = process_batch_resident(c, batch, adj, device=0)
        assert r["accepted"] == len(hs) and r["reject"] is None, r
        assert c.tip().hash == ref.tip().hash and c.height() == ref.height()
    assert r["device_ms"] > 0 and r["dgw_gpu"]


def _tampered(core, params, hs, i, field):
    act = params.kawpow_activation_time
    bad = [core.BlockHeader.deserialize(h.serialize(act), act) for h in hs]
    h = bad[i]
    if field == "mix":
        m = bytearray(h.mix_hash)
        m[3] ^= 1
        h.mix_hash = bytes(m)
    elif field == "nonce":
        h.nonce64 ^= 1 << 40
    elif field == "bits":
        h.bits ^= 1
    elif field == "solution":
        s = bytearray(h.solution)
        s[100] ^= 0x10
        h.solution = bytes(s)
    bad[i] = h
    return bad


@pytest.mark.parametrize("field,fixture,index", [("mix", "testnet_kawpow_10k.hdr", 4321),
                                                 ("nonce", "testnet_kawpow_10k.hdr", 9000),
                                                 ("bits", "testnet_kawpow_10k.hdr", 7000),
                                                 ("solution", "testnet_mixed_10k.hdr", None),
                                                 ("mix", "testnet_mixed_e384_10k.hdr", 8100)])
def test_resident_rejects_like_host(core, gpu, field, fixture, index):
    from nodexa_chain_core_amd.models.verify import process_batch_resident

    params, hs, _raw = _load(core, fixture)
    act = params.kawpow_activation_time
    if index is None:
        index = next(i for i in range(len(hs) - 1, 0, -1) if hs[i].is_equihash())
    bad = _tampered(core, params, hs, index, field)
    adj = hs[-1].time + 3600
    want = _chain(core, params, fixture).accept_headers(bad[:index + 1], adj, True)  # host golden PoW
    batch = core.HeaderBatch.from_headers(bad, act)
    c = _chain(core, params, fixture)
    r = process_batch_resident(c, batch, adj, device=0)
    assert r["accepted"] == len(want) - 1 == index, (r, want[-1].reject)
    assert r["reject"]["index"] == index and r["reject"]["reason"] == want[-1].reject


def test_resident_one_rank_rccl_gather(core, gpu, tmp_path):
    """The multi-rank form (slices + the RCCL all-gather of codes and hashes) on a forced one-rank
    process group: same result as the plain run."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = f"""
import sys, json
sys.path.insert(0, {root!r})
from nodexa_chain_core_amd import _core as core
from nodexa_chain_core_amd.models import synthetic
from nodexa_chain_core_amd.models.verify import process_batch_resident
from nodexa_chain_core_amd.parallel import world as W
w = W.init(use_gpu=True, force_collectives=True)
params, hs = synthetic.load({os.path.join(DATA, 'testnet_mixed_10k.hdr')!r})
batch = core.HeaderBatch.from_headers(list(hs), params.kawpow_activation_time)
c = core.HeaderChain(params)
r = process_batch_resident(c, batch, hs[-1].time + 3600, device=0, world=w)
print(json.dumps({{"accepted": r["accepted"], "backend": w.backend, "tip": core.u256_hex(c.tip().hash)}}))
W.shutdown()
"""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29500 + os.getpid() % 500), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    import json

    out = json.loads(r.stdout.strip().splitlines()[-1])
    params, hs, _ = _load(core, "testnet_mixed_10k.hdr")
    ref = core.HeaderChain(params)
    ref.accept_headers(hs, hs[-1].time + 3600, False)
    assert out["backend"] == "nccl" and out["accepted"] == len(hs) and out["tip"] == core.u256_hex(ref.tip().hash)
    assert np.all(True)


def test_wave_uniform_full_hashes_equal_lds_interpreter(core, gpu):
    """kawpow_verify_waves (wave-uniform programs, mix in VGPRs) against kawpow_verify_dag (the
    LDS-mix interpreter): the same digest and final hash for every KawPow row of the batch."""
    import torch

    from nodexa_chain_core_amd.models.verify import resident_verifier
    from nodexa_chain_core_amd.ops import header_batch as HB

    params, hs, raw = _load(core, "testnet_kawpow_10k.hdr")
    batch = core.HeaderBatch.from_bytes(raw, params.kawpow_activation_time)
    v = resident_verifier(0)
    plan = v.plan(batch)
    series = core.HeaderChain(params).dgw_ancestors(batch.header(0).prev)
    out = {}
    saved = HB.WAVES
    try:
        for waves in (False, True):
            HB.WAVES = waves
            if hasattr(v, "full"):
                v.full.zero_()
                torch.cuda.synchronize()
            r = v.run(params, batch, series, plan)
            torch.cuda.synchronize()
            out[waves] = (v.full[:len(hs) * 16].cpu().numpy().copy(), np.array(r["codes"]))
    finally:
        HB.WAVES = saved
    kp = np.flatnonzero(np.frombuffer(batch.kinds, np.uint8) == 0)
    a = out[False][0].reshape(-1, 16)[kp]
    b = out[True][0].reshape(-1, 16)[kp]
    assert (a == b).all(), int((a != b).any(1).sum())
    assert (out[False][1] == out[True][1]).all()


def test_p2p_header_sync_takes_the_resident_path(core, gpu, tmp_path):
    """nodexad -gpus=0 -p2pverifymode=dag syncing headers from a peer: every `headers` message goes
    through the device-resident pipeline (process_batch_resident) and the chain matches the peer's."""
    import time

    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.utils.config import ArgsManager
    from nodexa_chain_core_amd.utils.metrics import REGISTRY

    def node(name, extra):
        addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
        d = tmp_path / name
        d.mkdir()
        args = ArgsManager()
        args.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", f"-datadir={d}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                               f"-miningaddress={addr}", "-printtoconsole=0", *extra])
        n = Node(args)
        n.start()
        return n

    a = node("a", ["-listen", "-port=0"])
    b = None
    try:
        a.miner.generate(a.mining_script, 40)
        before = REGISTRY.counter("p2p_headers_resident_total")
        b = node("b", [f"-connect=127.0.0.1:{a.connman.port}", "-gpus=0", "-p2pverifymode=dag"])
        t = time.time() + 120
        while time.time() < t and b.state.chain.height() < 40:
            time.sleep(0.05)
        assert b.state.chain.height() == 40 and b.state.chain.tip().hash == a.state.chain.tip().hash
        assert REGISTRY.counter("p2p_headers_resident_total") - before >= 40
    finally:
        if b is not None:
            b.stop()
        a.stop()


def test_miner_dag_doubles_as_verify_epoch(core, gpu):
    """A mining node's DAG (miner/search.GpuSearchDevice) is offered to batch verify
    (ops/verify.share_epoch): resident_ready() then sends epoch-0 header batches down the resident
    path, and that path runs on the miner's own DAG tensor (no second build)."""
    from nodexa_chain_core_amd.miner.search import GpuSearchDevice
    from nodexa_chain_core_amd.models.verify import process_batch_resident, resident_ready
    from nodexa_chain_core_amd.ops import verify as V

    params, hs, raw = _load(core, "testnet_kawpow_10k.hdr")
    act = params.kawpow_activation_time
    V._epochs.pop((0, 0), None)
    dev = GpuSearchDevice(0)
    try:
        dev.searcher(5)  # builds (or reuses) epoch 0 for mining
        mined = dev.epochs[0]
        assert V._epochs.get((0, 0)) is mined
        batch_hs = hs[:2000]  # heights 1..2000: epoch 0 only
        assert resident_ready(batch_hs, act, 0, "auto")
        c = core.HeaderChain(params)
        r = process_batch_resident(c, core.HeaderBatch.from_headers(batch_hs, act), hs[-1].time + 3600, device=0)
        assert r["accepted"] == 2000 and r["reject"] is None
        assert V._epochs.get((0, 0)) is mined  # verify used it, built nothing of its own
    finally:
        dev.close()
