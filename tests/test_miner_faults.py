"""Miner failure handling on the one mining loop (miner/service.py): fault injection
(-gpufailrate / -dropshare) around the service's devices, eviction and re-partition in a gloo
world of 3, the hang watchdog, per-rank observability (getmininginfo.gpus[] has one entry per
rank), resume state and the metrics log. CPU devices over a regtest chain (KawPow from
genesis+1)."""
import json
import os
import time

import pytest

from test_miner_service import _check_disjoint, _run_world


@pytest.fixture()
def state(core):
    from nodexa_chain_core_amd.chain.state import REGTEST_KAWPOW_FROM_GENESIS, ChainState, make_params

    return ChainState(make_params("regtest", REGTEST_KAWPOW_FROM_GENESIS), None)


def test_gloo_world3_evicts_failing_rank_and_repartitions(tmp_path, core):
    """Rank 2's device fails every window (-gpufailrate=1): after 3 failed windows it is evicted,
    exits with EXIT_DEVICE_FAILED, and ranks 0-1 re-form the world and finish the blocks."""
    from nodexa_chain_core_amd.miner.service import EXIT_DEVICE_FAILED

    codes, outs, report = _run_world(tmp_path, 3, blocks=3, timeout_s=4.0,
                                     rank_env={2: {"NODEXA_MINER_FAILRATE": "1"}})
    assert codes[2] == EXIT_DEVICE_FAILED, "\n".join(outs)
    assert codes[0] == 0 and codes[1] == 0, "\n".join(outs)
    rep = json.load(open(report))
    assert rep["height"] == 6 and rep["world_size"] == 2 and rep["stats"]["bad_shares"] == 0
    # gpus[] listed every rank of the world of 3, with the failing rank's failures visible
    first = rep["gpus_first"]
    assert [g["rank"] for g in first] == [0, 1, 2]
    assert {"hashespersec", "stale_rate", "epochs_resident", "collective_ms", "last_device_ms",
            "aborted_workgroups", "failures"} <= set(first[0])
    assert len(rep["gpus_last"]) == 2 and all(g["hashes"] > 0 for g in rep["gpus_last"])
    r2 = json.load(open(tmp_path / "rank2.json"))
    assert r2["failures"] >= 3 and r2["hashes_total"] >= 0
    _check_disjoint(tmp_path, 3, rep)


def test_gloo_world8_shrinks_to_7(tmp_path, core):
    """The node's 8-rank shape (one rank per GPU of an MI355X node) with rank 5's device failing
    every window: the 8 ranks mine from disjoint nonce ranges, rank 5 is evicted, and the other 7
    re-form the world (8 -> 7) and finish the blocks; every share the node took re-checks on the host."""
    from nodexa_chain_core_amd.miner.service import EXIT_DEVICE_FAILED

    # 8 ranks on a loaded 8-CPU host start seconds apart: the default group's rendezvous has its
    # own generous timeout (world.rendezvous_timeout); the loop's collective timeout only has to
    # cover the shrunk group's connect (the failing rank exits, its peers see closed sockets)
    codes, outs, report = _run_world(tmp_path, 8, blocks=2, timeout_s=20.0,
                                     rank_env={5: {"NODEXA_MINER_FAILRATE": "1"}})
    assert codes[5] == EXIT_DEVICE_FAILED, "\n".join(outs)
    assert all(codes[r] == 0 for r in range(8) if r != 5), (codes, "\n".join(outs))
    rep = json.load(open(report))
    assert rep["height"] == 4 and rep["world_size"] == 7 and rep["stats"]["bad_shares"] == 0
    assert [g["rank"] for g in rep["gpus_first"]] == list(range(8))
    assert len(rep["gpus_last"]) == 7
    _check_disjoint(tmp_path, 8, rep)


def test_single_rank_all_failing_raises(state):
    from nodexa_chain_core_amd.miner.service import Miner

    m = Miner.local(state, fail_rate=1.0, max_failures=2)
    try:
        with pytest.raises(RuntimeError, match="evicted"):
            m.generate(bytes([0x51]), 1)
        info = m.service.rank_info()
        assert len(info) == 1 and info[0]["alive"] is False
    finally:
        m.close()


def test_dropshare_loses_every_share(state):
    from nodexa_chain_core_amd.miner.service import Miner

    m = Miner.local(state, drop_rate=1.0, window=64)
    try:
        assert m.generate(bytes([0x51]), 1, max_tries=200) == []
        assert m.service.dev.dropped > 0 and state.height() == 0
    finally:
        m.close()


def test_watchdog_stops_hung_single_rank(state):
    """A window that never finishes: the watchdog raises DeviceHung inside the loop, the service
    stops with the error and generate reports it instead of hanging."""
    from nodexa_chain_core_amd.miner.search import CpuSearchDevice, HangingDevice, RankDevice
    from nodexa_chain_core_amd.miner.service import ChainLeader, Miner, MiningService

    dev = HangingDevice(RankDevice(CpuSearchDevice(max_window=8)), after=0)
    svc = MiningService(dev, ChainLeader(state), window=8, watchdog_s=0.5).start()
    m = Miner(state, svc)
    try:
        t0 = time.time()
        with pytest.raises(RuntimeError, match="hang"):
            m.generate(bytes([0x51]), 1)
        assert time.time() - t0 < 20 and isinstance(svc.error, Exception)
    finally:
        m.close()


def test_resume_state_continues_extranonce(state, tmp_path):
    from nodexa_chain_core_amd import core
    from nodexa_chain_core_amd.miner.service import ChainLeader

    _core = core()
    path = str(tmp_path / "miner_state.json")
    a = ChainLeader(state, state_path=path)
    a.mine(bytes([0x51]))
    for _ in range(5):
        a.next_work(repartitioned=True)  # five jobs on the same tip: extranonce 1..5
    saved = json.load(open(path))
    assert saved["extranonce"] == 5 and saved["tip"] == _core.u256_hex(state.tip().hash)
    b = ChainLeader(state, state_path=path)  # a restart on the same tip
    b.mine(bytes([0x51]))
    b.next_work()
    job = next(reversed(b.jobs.values()))
    sig = job.block.vtx[0].vin[0].script_sig
    assert sig.endswith(_core.script_push_data(_core.scriptnum(6)))  # continues, never re-searches 1..5
    assert json.load(open(path))["extranonce"] == 6


def test_node_metrics_log_and_rest(core, tmp_path):
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.utils import metrics
    from nodexa_chain_core_amd.utils.config import ArgsManager

    metrics.REGISTRY.reset()
    addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
    args = ArgsManager()
    args.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
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
        assert len(info["gpus"]) == 1 and info["gpus"][0]["blocks"] == 2 and info["gpus"][0]["algo"] == "kawpow"
        assert core.light_cache_dir().endswith("dagcache")
        core.create_epoch_context(0)  # (epoch 0 may already sit in the in-process LRU)
    finally:
        n.stop()
        core.set_light_cache_dir("")
    lines = [json.loads(x) for x in open(os.path.join(n.datadir, "metrics.jsonl"))]
    names = {c["name"] for c in lines[-1]["counters"]}
    assert {"miner_hashes_total", "miner_shares_total", "miner_blocks_total"} <= names
    assert [f for f in os.listdir(os.path.join(n.datadir, "dagcache")) if f.startswith("light-0-")]
    assert json.load(open(os.path.join(n.datadir, "miner_state.json")))["extranonce"] >= 1
