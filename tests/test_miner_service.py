"""The node's mining loop (miner/search.py + miner/service.py) on CPU devices.

* single rank: the pipelined loop mines regtest blocks that ProcessNewBlock accepts, a stale
  window is aborted by the generation word, shares are fully re-hashed before use;
* gloo worlds of 2 and 4 processes (rank 0 = chain + leader, ranks >= 1 = followers): blocks
  found across ranks, a template change mid-run (tip changes and a new coinbase script), and no
  nonce window searched twice within a job;
* rank failure: one follower's device hangs mid-search inside the loop; it exits with
  EXIT_DEVICE_HUNG, the survivors rebuild the group without it and keep mining.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def state(core):
    from nodexa_chain_core_amd.chain.state import REGTEST_KAWPOW_FROM_GENESIS, ChainState, make_params

    return ChainState(make_params("regtest", REGTEST_KAWPOW_FROM_GENESIS), None)


def test_work_packet_roundtrip():
    from nodexa_chain_core_amd.miner.search import ALGO_EQUIHASH, FLAG_CLEAN, WORK_SIZE, Work

    w = Work(bytes(range(32)), bytes([0x7F] + [0xFF] * 31), 7500 * 3 + 5, 42, 1 << 56, FLAG_CLEAN)
    raw = w.pack()
    assert len(raw) == WORK_SIZE == 144
    back = Work.unpack(raw)
    assert back == w and back.epoch == 3 and not back.idle and back.target64() == 0x7FFFFFFFFFFFFFFF
    assert back.header_hash == bytes(range(32)) and back.algo == 0
    assert Work().idle and Work.unpack(Work().pack()).idle
    e = Work(bytes(range(80)), bytes(32), 9, 3, 0, 0, ALGO_EQUIHASH)  # the 80-byte Equihash prefix
    assert Work.unpack(e.pack()) == e and Work.unpack(e.pack()).header == bytes(range(80))


def test_record_roundtrip():
    from nodexa_chain_core_amd.miner.search import ALGO_EQUIHASH, ALGO_X16RV2, EquihashShare, LegacyShare, SlotResult
    from nodexa_chain_core_amd.miner.service import (MAX_SHARES, MAX_SHARES_PER_STEP, RECORD_SIZE, pack_record,
                                                     unpack_record)
    from nodexa_chain_core_amd.ops.kawpow import Share

    shares = [Share(i, bytes([i]) * 32, bytes([255 - i]) * 32) for i in range(MAX_SHARES_PER_STEP + 3)]
    raw = pack_record(SlotResult(9, 100, 4096, 4000, shares, 12.5, 7), coll_ms=0.25, failures=1, epochs=[3, 4],
                      device=5)
    assert len(raw) == RECORD_SIZE
    rec = unpack_record(raw)
    assert (rec.job_id, rec.hashes) == (9, 4000) and rec.shares == shares[:MAX_SHARES_PER_STEP]
    assert (rec.device_ms, rec.aborted, rec.coll_ms, rec.failures, rec.epochs, rec.device) == (12.5, 7, 0.25, 1, [3, 4], 5)
    assert rec.has_result and rec.alive
    empty = unpack_record(pack_record(None, alive=False))
    assert (empty.job_id, empty.hashes, empty.shares, empty.has_result, empty.alive) == (0, 0, [], False, False)
    eq = [EquihashShare(i, bytes([i]) * 1344, bytes([i + 1]) * 32) for i in range(6)]
    back = unpack_record(pack_record(SlotResult(2, 0, 16, 31, eq, 8.0, 0, ALGO_EQUIHASH)))
    assert back.algo == ALGO_EQUIHASH and back.hashes == 31 and back.shares == eq[:MAX_SHARES[ALGO_EQUIHASH]]
    lg = [LegacyShare(7, bytes(32))]
    assert unpack_record(pack_record(SlotResult(4, 0, 65536, 8, lg, 1.0, 0, ALGO_X16RV2))).shares == lg


def test_record_totals_replace_the_counter_all_reduce():
    """The step's hash counter and next-epoch votes ride in the gathered records: every rank sums
    them from the all-gather (one collective less per step than an all-reduce of their own)."""
    from nodexa_chain_core_amd.miner.search import SlotResult
    from nodexa_chain_core_amd.miner.service import pack_record, record_totals

    recs = [pack_record(SlotResult(1, 0, 4096, 4096, [], 1.0), vote=True),
            pack_record(None, vote=True),
            pack_record(SlotResult(1, 4096, 4096, 4000, [], 1.0), vote=False)]
    assert record_totals(recs) == (8096, 2)
    assert record_totals([pack_record(None)]) == (0, 0)


def test_single_rank_loop_mines_blocks(state):
    from nodexa_chain_core_amd.miner.search import CpuSearchDevice
    from nodexa_chain_core_amd.miner.service import ChainLeader, MiningService

    leader = ChainLeader(state, target_bits=4)
    svc = MiningService(CpuSearchDevice(max_window=8), leader, window=8, record_windows=True)
    req = leader.mine(bytes([0x51]), blocks=3)
    for _ in range(400):
        if req.done.is_set():
            break
        svc.step()
    assert req.done.is_set() and req.error is None
    assert len(req.found) == 3 and state.height() == 3
    assert leader.stats["blocks"] == 3 and leader.stats["bad_shares"] == 0
    assert svc.hashes_total > 0 and req.tries == svc.hashes_total
    # windows of one job never overlap (single rank: consecutive cursors)
    by_job = {}
    for job, start, count in svc.windows:
        by_job.setdefault(job, []).append((start, count))
    for wins in by_job.values():
        wins.sort()
        assert all(a[0] + a[1] <= b[0] for a, b in zip(wins, wins[1:]))
    # idle packet afterwards: the loop drains and keeps stepping without a request
    assert svc.step() and svc.work.idle


def test_loop_background_thread_and_stop(state):
    from nodexa_chain_core_amd.miner.search import CpuSearchDevice
    from nodexa_chain_core_amd.miner.service import ChainLeader, MiningService

    leader = ChainLeader(state, target_bits=3)
    svc = MiningService(CpuSearchDevice(max_window=8), leader, window=8).start()
    try:
        req = leader.mine(bytes([0x51]), blocks=2)
        assert req.done.wait(60) and len(req.found) == 2
        assert svc.hashrate() >= 0
    finally:
        svc.stop()
    assert svc._thread is None and svc.error is None


def test_abort_drops_stale_window(state):
    from nodexa_chain_core_amd.miner.search import CpuSearchDevice, SearchPipeline, Work

    dev = CpuSearchDevice(max_window=4)
    pipe = SearchPipeline(dev)
    w = Work(bytes(32), bytes([0x7F] + [0xFF] * 31), 1, 1, 0, 0)
    assert pipe.step(w, 0, 4) is None
    dev.abort()  # the template changed while window 0 was queued
    res = pipe.step(w, 4, 4)
    assert res.hashes == 0 and res.shares == []
    res = pipe.drain()
    assert res.hashes > 0 and res.shares  # window 1 was queued after the abort: it runs


def test_leader_rejects_share_failing_full_rehash(state):
    from nodexa_chain_core_amd.miner.service import ChainLeader
    from nodexa_chain_core_amd.ops.kawpow import Share

    leader = ChainLeader(state, target_bits=0)
    req = leader.mine(bytes([0x51]), blocks=1)
    w = leader.next_work()
    from nodexa_chain_core_amd import core

    _core = core()
    ctx = _core.get_epoch_context(0)
    ok, nonce, fin, mix = _core.kawpow_search_light(ctx, w.height, w.header_hash, w.boundary, 0, 100)
    assert ok
    bad_mix = bytes([mix[0] ^ 1]) + mix[1:]
    # a share whose final hash is right but whose mix is not (a wrong DAG gather would look like
    # this after the mix-only check) is dropped by the full re-hash
    leader.on_results([(w.job_id, 10, [Share(nonce, bad_mix, fin)])])  # (job, hashes, shares) tuples work too
    assert leader.stats["bad_shares"] == 1 and state.height() == 0 and not req.done.is_set()
    leader.on_results([(w.job_id, 10, [Share(nonce, mix, fin)])])
    assert state.height() == 1 and req.done.is_set() and len(req.found) == 1


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_world(tmp_path, n, blocks=2, hang_rank=None, timeout_s=8.0, extra_env=None, rank_env=None):
    port = _free_port()
    procs = []
    base = dict(os.environ)
    base.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(n),
                 "NODEXA_MINER_CPU": "1", "NODEXA_MINER_WINDOW": "8", "NODEXA_TEST_BLOCKS": str(blocks),
                 "NODEXA_MINER_COLLECTIVE_TIMEOUT": str(timeout_s), "NODEXA_MINER_WATCHDOG": "3",
                 "PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1"})
    base.update(extra_env or {})
    report = tmp_path / "rank0.json"
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        env["NODEXA_MINER_WINDOWS_LOG"] = str(tmp_path / f"rank{r}.json")
        if r == hang_rank:
            env["NODEXA_MINER_HANG_AFTER"] = "3"
        env.update((rank_env or {}).get(r, {}))
        if r == 0:
            cmd = [sys.executable, os.path.join(ROOT, "tests", "miner_world_rank0.py"), str(report)]
        else:
            cmd = [sys.executable, "-m", "nodexa_chain_core_amd.miner.service"]
        procs.append(subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    codes, outs = [], []
    deadline = time.time() + 280
    for p in procs:
        try:
            out, _ = p.communicate(timeout=max(1.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        codes.append(p.returncode)
        outs.append(out.decode(errors="replace"))
    return codes, outs, report


def _check_disjoint(tmp_path, n, rep):
    windows = [(0, *w) for w in rep["windows"]]
    for r in range(1, n):
        path = tmp_path / f"rank{r}.json"
        if path.exists():
            windows += [(r, *w) for w in json.load(open(path))["windows"]]
    by_job = {}
    for r, job, start, count in windows:
        by_job.setdefault(job, []).append((start, start + count, r))
    multi = 0
    for job, ivs in by_job.items():
        ivs.sort()
        multi += len({r for *_x, r in ivs}) > 1
        for a, b in zip(ivs, ivs[1:]):
            assert a[1] <= b[0], f"job {job}: windows {a} and {b} overlap"
    return multi


@pytest.mark.parametrize("n", [2, 4])
def test_gloo_world_mines_with_template_change(tmp_path, core, n):
    codes, outs, report = _run_world(tmp_path, n, blocks=2)
    assert codes == [0] * n, "\n".join(outs)
    rep = json.load(open(report))
    assert rep["height"] == 4 and [len(f) for f in rep["found"]] == [2, 2]
    # the request switched coinbase scripts mid-run: every block pays the script that was current
    assert rep["coinbase"] == [["51", "51"], ["52", "52"]]
    assert rep["stats"]["bad_shares"] == 0 and rep["world_size"] == n
    # every rank searched (hashes all-reduced into rank 0's counter, per-rank records gathered)
    assert len(rep["rank_hashes"]) == n and all(int(v) > 0 for v in rep["rank_hashes"].values())
    assert rep["hashes_total"] == sum(int(v) for v in rep["rank_hashes"].values())
    assert _check_disjoint(tmp_path, n, rep) > 0  # jobs searched by several ranks, never twice


def test_gloo_world_survives_hung_rank(tmp_path, core):
    n = 3
    codes, outs, report = _run_world(tmp_path, n, blocks=3, hang_rank=2, timeout_s=4.0)
    from nodexa_chain_core_amd.miner.service import EXIT_DEVICE_HUNG

    assert codes[2] == EXIT_DEVICE_HUNG, "\n".join(outs)
    assert codes[0] == 0 and codes[1] == 0, "\n".join(outs)
    rep = json.load(open(report))
    assert rep["height"] == 6 and rep["world_size"] == 2  # re-formed without the hung rank
    assert rep["stats"]["bad_shares"] == 0
    r1 = json.load(open(tmp_path / "rank1.json"))
    assert r1["world_size"] == 2 and r1["rank"] == 1
    _check_disjoint(tmp_path, n, rep)


def test_node_mines_through_service_with_follower_rank(core, tmp_path):
    """nodexad -minerservice -minerranks=2: the node is rank 0 of a gloo world and spawns rank 1
    itself; generate / setgenerate / getmininginfo go through the service."""
    from nodexa_chain_core_amd.node import Node
    from nodexa_chain_core_amd.rpc.client import RPCClient
    from nodexa_chain_core_amd.utils.config import ArgsManager

    addr = core.base58check_encode(bytes([42]) + bytes(range(20)))
    args = ArgsManager()
    args.parse_parameters(["-regtest", "-kawpowactivationtime=1524179367", f"-datadir={tmp_path}", "-rpcport=0", "-rpcuser=u", "-rpcpassword=p",
                           f"-miningaddress={addr}", "-printtoconsole=0", "-minerservice", "-minerranks=2",
                           "-gpuintensity=8", "-minertargetbits=5", "-minercollectivetimeout=20"])
    n = Node(args)
    n.start()
    try:
        c = RPCClient("127.0.0.1", n.rpc.port, "u", "p")
        hashes = c.generatetoaddress(3, addr)
        assert len(hashes) == 3 and c.getblockcount() == 3
        assert n.miner.service.world_size == 2 and len(n.miner_procs) == 1
        c.setgenerate(True)
        assert c.getgenerate() is True
        deadline = time.time() + 120
        while c.getblockcount() < 5 and time.time() < deadline:
            time.sleep(0.2)
        info = c.getmininginfo()
        assert c.getblockcount() >= 5 and info["hashespersec"] > 0
        assert [w["worker"] for w in info["workers"]] == [0, 1] and all(w["hashes"] > 0 for w in info["workers"])
        c.setgenerate(False)
        assert c.getgenerate() is False
    finally:
        n.stop()
    assert [p.returncode for p in n.miner_procs] == [0]
