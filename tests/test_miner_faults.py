"""Miner failure handling: fault injection (-gpufailrate / -dropshare),
eviction + nonce re-partition, the hang watchdog, resume state and the metrics log.
All on CPU backends over a regtest chain (KawPow from genesis+1)."""
import json
import threading
import time

import pytest


@pytest.fixture()
def state(core):
    from nodexa_chain_core_amd.chain.state import ChainState, make_params

    return ChainState(make_params("regtest"), None)


def _controller(state, backends, **kw):
    from nodexa_chain_core_amd.miner.kawpow_miner import MinerController

    return MinerController(state, backends, **kw)


def test_fault_eviction_and_repartition(state):
    from nodexa_chain_core_amd.miner.kawpow_miner import CpuKawpowBackend, FaultInjector

    bad = FaultInjector(CpuKawpowBackend(), fail_rate=1.0, seed=1)
    ok = CpuKawpowBackend()
    m = _controller(state, [bad, ok], max_failures=3)
    assert m.nonce_base(1) == 1 << 56
    hashes = m.generate(bytes([0x51]), 3)
    assert len(hashes) == 3 and state.height() == 3
    assert not m.health[0].alive and m.health[0].total_failures == 3
    assert m.health[1].alive and m.health[1].blocks == 3
    assert m.nonce_base(1) == 0  # survivor re-ranked to the start of the nonce space
    assert m.metrics.counter("miner_evictions_total", worker=m.health[0].label) >= 1


def test_all_backends_failing_raises(state):
    from nodexa_chain_core_amd.miner.kawpow_miner import CpuKawpowBackend, FaultInjector

    m = _controller(state, [FaultInjector(CpuKawpowBackend(), fail_rate=1.0)], max_failures=2)
    with pytest.raises(RuntimeError, match="evicted"):
        m.generate(bytes([0x51]), 1)


def test_dropshare_loses_every_share(state):
    from nodexa_chain_core_amd.miner.kawpow_miner import CpuKawpowBackend, FaultInjector

    be = FaultInjector(CpuKawpowBackend(), drop_rate=1.0)
    m = _controller(state, [be])
    assert m.generate(bytes([0x51]), 1, max_tries=200) == []
    assert be.dropped > 0 and state.height() == 0


class _HangingBackend:
    name = "hang"
    device = 7

    def __init__(self):
        self.release = threading.Event()

    def search(self, *a):
        self.release.wait(30)
        return None


def test_watchdog_evicts_hung_worker(state):
    from nodexa_chain_core_amd.miner.kawpow_miner import CpuKawpowBackend

    hang = _HangingBackend()
    m = _controller(state, [hang, CpuKawpowBackend()], watchdog_s=0.5)
    m.set_generate(True, bytes([0x51]))
    try:
        deadline = time.time() + 20
        while m.health[0].alive and time.time() < deadline:
            time.sleep(0.1)
        assert not m.health[0].alive and "hung" in m.health[0].last_error
        while state.height() < 2 and time.time() < deadline:
            time.sleep(0.1)
        assert state.height() >= 2  # the healthy worker kept mining
    finally:
        hang.release.set()
        m.stop()


def test_resume_state_continues_extranonce(state, tmp_path):
    from nodexa_chain_core_amd.miner.kawpow_miner import CpuKawpowBackend

    path = str(tmp_path / "miner_state.json")
    m = _controller(state, [CpuKawpowBackend()], state_path=path)
    tip = state.tip()
    from nodexa_chain_core_amd import core

    tip_hex = core().u256_hex(tip.hash)
    m._set_cursor(0, tip_hex, 17, 12345)
    m.save_state()
    m2 = _controller(state, [CpuKawpowBackend()], state_path=path)
    assert m2.resume_extranonce(0, tip_hex) == 17
    assert m2.resume_extranonce(0, "00" * 32) == 0
    assert json.load(open(path))["workers"]["0"]["cursor"] == 12345


def test_node_metrics_log_and_rest(core, tmp_path):
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.utils import metrics
    from nodexa_chain_core_amd.utils.config import ArgsManager

    metrics.REGISTRY.reset()
    addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
    args = ArgsManager()
    args.parse_parameters(["-regtest", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                           f"-miningaddress={addr}", "-printtoconsole=0", "-metricslog=metrics.jsonl",
                           "-metricsinterval=60", "-dagcache=1"])
    n = Node(args)
    n.start()
    try:
        n.miner.generate(n.mining_script, 2)
        code, _, body = n.rest("/rest/metrics")
        assert code == 200 and b"nodexa_miner_blocks_total" in body
        info = n.table.execute("getmininginfo", [])
        assert info["workers"][0]["blocks"] == 2
        assert core.light_cache_dir().endswith("dagcache")
        core.create_epoch_context(0)  # (epoch 0 may already sit in the in-process LRU)
    finally:
        n.stop()
        core.set_light_cache_dir("")
    import os

    lines = [json.loads(x) for x in open(os.path.join(n.datadir, "metrics.jsonl"))]
    names = {c["name"] for c in lines[-1]["counters"]}
    assert {"miner_hashes_total", "miner_shares_total", "miner_blocks_total"} <= names
    assert [f for f in os.listdir(os.path.join(n.datadir, "dagcache")) if f.startswith("light-0-")]
