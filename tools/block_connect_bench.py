"""Block connection throughput: ConnectBlock of a synthetic payments block (one signed P2PKH /
P2WPKH spend per transaction) with host script checks on 1 and T threads (the reference's
CCheckQueue model, -par) versus deferred signatures verified in one GPU batch
(ops/secp.verify_batch). Prints one JSON line per mode; the view is restored with
DisconnectBlock between runs (not timed).

    python tools/block_connect_bench.py --txs 8000 --threads 16 --reps 3
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nodexa_chain_core_amd import _core  # noqa: E402
from nodexa_chain_core_amd.utils.synth_block import make_signed_block  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txs", type=int, default=8000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args()
    t0 = time.time()
    blk, view, height = make_signed_block(a.txs, seed=11, witness_every=4)
    print(f"built {a.txs}-tx block in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    flags = _core.BLOCK_SCRIPT_VERIFY_FLAGS

    def run(threads, defer, verify=None):
        best = None
        for _ in range(a.reps):
            t = time.perf_counter()
            res, undo = _core.connect_block(blk, height, view, True, defer, None, 0, flags, threads)
            assert res.ok, res.reject
            if verify is not None:
                v = verify(res.sig_items())
                assert all(v), "GPU batch rejected a valid signature"
            dt = time.perf_counter() - t
            assert _core.disconnect_block(blk, undo, view)
            best = dt if best is None else min(best, dt)
        return best

    modes = [("host_serial", 1, False, None), (f"host_par{a.threads}", a.threads, False, None)]
    if a.gpu:
        import torch

        from nodexa_chain_core_amd.ops import secp

        torch.cuda.init()
        secp.verify_batch(blk and [( _core.secp_pubkey_create(b"\x01" * 32, True), b"\x30\x06\x02\x01\x01\x02\x01\x01",
                                     bytes(32))])  # warm the module / comb table
        modes.append((f"gpu_batch_par{a.threads}", a.threads, True, secp.verify_batch))
    base = None
    for name, threads, defer, verify in modes:
        dt = run(threads, defer, verify)
        base = base or dt
        print(json.dumps({"mode": name, "txs": a.txs, "ms": round(dt * 1e3, 2),
                          "inputs_per_s": round(a.txs / dt), "speedup_vs_serial": round(base / dt, 2)}), flush=True)


if __name__ == "__main__":
    main()
