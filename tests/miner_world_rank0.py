"""Rank 0 of a multi-process mining world for tests/test_miner_service.py (gloo, CPU devices).

Runs a regtest ChainState with the ChainLeader and mines `NODEXA_TEST_BLOCKS` blocks to one
script, then switches the request to a second script (a template change that is not a tip
change) for as many more, then sends the stop packet. Writes a JSON report to argv[1].
NODEXA_TEST_EQUIHASH=1: the chain's Equihash extension is active from now on, so every block is
an Equihash(200,9) block mined by the ranks' golden solvers."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_path: str) -> int:
    from nodexa_chain_core_amd import core
    from nodexa_chain_core_amd.chain.state import REGTEST_KAWPOW_FROM_GENESIS, ChainState, make_params
    from nodexa_chain_core_amd.miner.service import ChainLeader, MiningService, make_rank_device
    from nodexa_chain_core_amd.parallel import world as W

    _core = core()
    timeout = float(os.environ.get("NODEXA_MINER_COLLECTIVE_TIMEOUT", "30"))
    W.init(use_gpu=False, timeout_s=max(int(timeout), W.rendezvous_timeout()))
    blocks = int(os.environ.get("NODEXA_TEST_BLOCKS", "2"))
    window = int(os.environ.get("NODEXA_MINER_WINDOW", "8"))
    eq_act = int(time.time()) - 100 if os.environ.get("NODEXA_TEST_EQUIHASH") == "1" else None
    state = ChainState(make_params("regtest", REGTEST_KAWPOW_FROM_GENESIS, equihash_activation_time=eq_act), None)
    leader = ChainLeader(state, target_bits=int(os.environ.get("NODEXA_TEST_TARGET_BITS", "7")))
    dev = make_rank_device(True, window=window, fail_rate=float(os.environ.get("NODEXA_MINER_FAILRATE", "0")))
    svc = MiningService(dev, leader, window=window, collective_timeout_s=timeout, record_windows=True)
    scripts = [bytes([0x51]), bytes([0x52])]
    found, t0 = [], time.time()
    gpus_first = None
    for spk in scripts:
        req = leader.mine(spk, blocks=blocks)
        while not req.done.is_set():
            if time.time() - t0 > 240:
                raise SystemExit("rank 0: mining took too long")
            try:
                svc.step()
                if gpus_first is None and svc.steps >= 3:
                    gpus_first = svc.rank_info()  # getmininginfo.gpus[] of the full world
            except Exception as e:  # noqa: BLE001 — a lost rank: rebuild the world and go on
                from nodexa_chain_core_amd.miner.service import CollectiveError

                if not isinstance(e, CollectiveError):
                    raise
                svc.recover(e)
        found.append(list(req.found))
    leader.shutdown()
    while svc.step():
        pass
    act = state.params.kawpow_activation_time
    coinbase = [[_core.Block.deserialize(state.get_block_raw(_core.u256_from_hex(h)), act).vtx[0].vout[0]
                 .script_pubkey.hex() for h in hs] for hs in found]
    report = {"coinbase": coinbase, "height": state.height(), "found": found, "windows": svc.windows, "world_size": svc.world_size,
              "hashes_total": svc.hashes_total, "stats": leader.stats, "steps": svc.steps,
              "tip": _core.u256_hex(state.tip().hash), "rank_hashes": svc.rank_hashes,
              "gpus_first": gpus_first, "gpus_last": svc.rank_info(), "per_rank": leader.per_rank,
              "equihash_blocks": sum(1 for hs in found for h in hs
                                     if _core.Block.deserialize(state.get_block_raw(_core.u256_from_hex(h)), act)
                                     .header.is_equihash())}
    with open(out_path, "w") as f:
        json.dump(report, f)
    W.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
