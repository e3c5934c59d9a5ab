"""nodexad -gpus=0 on one MI355X: the node mines through its mining service (pipelined 2^25-nonce
windows, device-side stale-work abort, full share re-hash), getmininginfo reports the service's
rate per rank, every block it finds is accepted by ProcessNewBlock, and the rate it SUSTAINS over
more than 10 s of setgenerate is within 10 % of the bare kernel's on the same DAG.

`-minertargetbits=28` makes the miner search for hashes below 2^228 although regtest accepts
almost any hash: a block then takes ~2^28 hashes (about a second at full rate), so the loop runs
whole windows and pays its template changes (a new job and a stale-window abort per block) the way
a mining node does. The headline epoch (384, 4 GiB DAG) cannot be reached by a regtest chain, so
the same loop is also held there with a fixed job for over 10 s and compared with the kernel."""
import time

import pytest

pytestmark = pytest.mark.gpu


def _kernel_rate(core, epoch: int, window: int = 1 << 25) -> float:
    """The bare search kernel on this epoch's DAG: one window timed with device events."""
    import torch

    from nodexa_chain_core_amd.miner.search import GpuSearchDevice, Work

    dev = GpuSearchDevice(0)
    height = epoch * core.EPOCH_LENGTH + (123 if epoch else 5)  # periods build() ships kernels for
    s = dev.searcher(height)
    n = window // s.block * s.block
    hh = core.sha256d(b"kernel-rate")
    s.launch(hh, 0, n, 0)  # warm
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    s.launch(hh, n, n, 0)
    e1.record()
    e1.synchronize()
    rate = n / (e0.elapsed_time(e1) / 1e3)
    dev.close()
    del dev, Work
    torch.cuda.empty_cache()
    return rate


def test_node_setgenerate_sustains_kernel_rate(core, gpu, tmp_path):
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.rpc.client import RPCClient
    from nodexa_chain_core_amd.utils.config import ArgsManager

    kernel = _kernel_rate(core, 0)
    addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
    args = ArgsManager()
    args.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                           f"-miningaddress={addr}", "-printtoconsole=0", "-gpus=0", "-minertargetbits=28"])
    n = Node(args)
    n.start()
    try:
        c = RPCClient("127.0.0.1", n.rpc.port, "u", "p", timeout=300)
        assert c.generatetoaddress(1, addr, 1 << 40) and c.getblockcount() == 1  # DAG build + first block
        svc = n.miner.service
        c.setgenerate(True)
        time.sleep(2.0)  # past the first template
        h0, t0 = svc.hashes_total, time.perf_counter()
        time.sleep(12.0)
        h1, t1 = svc.hashes_total, time.perf_counter()
        info = c.getmininginfo()
        c.setgenerate(False)
        sustained = (h1 - h0) / (t1 - t0)
        assert sustained >= 0.9 * kernel, (sustained / 1e6, kernel / 1e6, info)
        assert c.getblockcount() >= 4
        g = info["gpus"][0]
        assert info["gpus"] and g["epochs_resident"] == [0] and g["algo"] == "kawpow" and g["hashespersec"] > 0
        assert g["last_device_ms"] > 0 and g["blocks"] >= 1 and info["hashespersec"] > 0.5 * kernel
        assert n.miner.service.leader.stats["bad_shares"] == 0
        assert c.verifychain(4, 0) is True
        # every mined header carries a valid KawPow proof for its own nNonce64 / mix
        for h in range(1, c.getblockcount() + 1):
            blk = c.getblock(c.getblockhash(h))
            nonce = blk["nonce64"] if isinstance(blk["nonce64"], int) else int(blk["nonce64"], 16)
            res = c.getkawpowhash(blk["headerhash"], blk["mixhash"], "%016x" % nonce, h)
            assert res["result"] == "true", (h, res)
    finally:
        n.stop()


def test_service_sustains_kernel_rate_at_headline_epoch(core, gpu):
    """Epoch 384 (4 GiB DAG): the mining loop with a fixed job for > 10 s against the bare kernel."""
    from nodexa_chain_core_amd.chain.header import BlockHeader
    from nodexa_chain_core_amd.miner.search import GpuSearchDevice, Work
    from nodexa_chain_core_amd.miner.service import BenchLeader, MiningService

    kernel = _kernel_rate(core, 384)
    height = 384 * core.EPOCH_LENGTH + 123
    hdr = BlockHeader(version=0x20000000, prev=core.sha256d(b"p"), merkle_root=core.sha256d(b"m"), time=1_700_000_000,
                      bits=0x1b00ffff, height=height)
    boundary = ((1 << 256) // (1 << 24) - 1).to_bytes(32, "big")
    dev = GpuSearchDevice(0)
    leader = BenchLeader(Work(hdr.progpow_header_hash(), boundary, height, 1, 0, 0))
    svc = MiningService(dev, leader, window=1 << 25)
    for _ in range(3):
        svc.step()
    h0, t0 = svc.hashes_total, time.perf_counter()
    while time.perf_counter() - t0 < 10.5:
        svc.step()
    h1, t1 = svc.hashes_total, time.perf_counter()
    leader.shutdown()
    while svc.step():
        pass
    svc.pipe.drain()
    sustained = (h1 - h0) / (t1 - t0)
    assert sustained >= 0.9 * kernel, (sustained / 1e6, kernel / 1e6)
    ctx = core.get_epoch_context(384)
    assert leader.shares and all(s.verify_full(height, leader.work.header_hash, boundary, ctx=ctx)
                                 for s in leader.shares[:4])
    dev.close()
