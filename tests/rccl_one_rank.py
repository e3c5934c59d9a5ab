"""One-rank RCCL world on one MI355X (tests/test_gpu_rccl.py runs this as a fresh process).

parallel/world.init(force_collectives=True) makes a real "nccl" (= RCCL) process group of one
rank, so every collective the 8-GPU node issues runs here too, as RCCL kernels on the device:
the sharded DAG build's in-place all_gather_into_tensor (parallel/dag.py), batch verify's result
all-gather (parallel/verify.py), and the mining loop's record all-gather / counter all-reduce /
work-packet broadcast on the loop's own communicator and stream (miner/service.Comm). Then a
collective failure is injected (NODEXA_MINER_FAIL_COLLECTIVE_AT): the loop's recover() aborts
its RCCL communicator (ncclCommAbort through _abort_process_group), makes a new one and mines on.
Writes a JSON report to argv[1]."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_path: str) -> int:
    import torch

    from nodexa_chain_core_amd import _build, core
    from nodexa_chain_core_amd.chain.header import BlockHeader
    from nodexa_chain_core_amd.miner.search import GpuSearchDevice, Work
    from nodexa_chain_core_amd.miner.service import BenchLeader, CollectiveError, MiningService
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import verify_headers
    from nodexa_chain_core_amd.parallel import world as W
    from nodexa_chain_core_amd.parallel.verify import verify_headers_distributed

    _build.build_all()
    _core = core()
    w = W.init(use_gpu=True, force_collectives=True, timeout_s=60)
    rep = {"backend": w.backend, "world_size": w.world_size, "collective": w.collective}
    assert w.backend == "nccl" and w.world_size == 1 and w.collective
    # 1. sharded DAG build: build(shard=(0, 1)) + in-place all_gather_into_tensor over RCCL
    dev = GpuSearchDevice(w.device.index, collective_dag=True)
    height = 123
    t0 = time.time()
    block = dev.searcher(height).block  # the L1 self-check runs on the gathered DAG
    torch.cuda.synchronize()
    rep["dag_s"] = round(time.time() - t0, 3)
    # 2. the mining loop on its own RCCL communicator
    hdr = BlockHeader(version=0x20000000, prev=_core.sha256d(b"rccl-prev"), merkle_root=_core.sha256d(b"rccl-m"),
                      time=1_700_000_000, bits=0x1b00ffff, height=height)
    boundary = ((1 << 256) // (1 << 20) - 1).to_bytes(32, "big")
    leader = BenchLeader(Work(hdr.progpow_header_hash(), boundary, height, 1, 0, 0))
    svc = MiningService(dev, leader, window=block * 4096, collective_timeout_s=30)
    assert svc.comm.active and svc.comm.gpu
    for _ in range(6):
        svc.step()
    rep["steps_before_abort"] = svc.steps
    rep["hashes_before_abort"] = svc.hashes_total
    # 3. an injected collective failure: abort the RCCL communicator, re-form, continue
    svc.comm.fail_at_step = svc.comm.calls + 1
    try:
        svc.step()
        rep["injected"] = False
    except CollectiveError as e:
        rep["injected"] = str(e)
        svc.recover(e)
    old_group = id(svc.comm.group)
    for _ in range(6):
        svc.step()
    rep["group_replaced"] = id(svc.comm.group) != old_group or rep["injected"] is not False
    rep["steps_after_abort"] = svc.steps
    rep["hashes_total"] = svc.hashes_total
    leader.shutdown()
    while svc.step():
        pass
    svc.pipe.drain()
    ctx = _core.get_epoch_context(0)
    bad = sum(not s.verify_full(height, leader.work.header_hash, boundary, ctx=ctx) for s in leader.shares[:8])
    rep["shares_checked"] = min(8, len(leader.shares))
    rep["share_mismatches"] = bad
    # 4. batch verify with the RCCL result all-gather == the plain path
    params, headers = synthetic.load(os.path.join(ROOT, "tests", "data", "testnet_kawpow_10k.hdr"))
    batch = headers[:2000]
    a = verify_headers_distributed(params, batch, mode="light")
    b = verify_headers(params, batch, gpus=[w.device.index], mode="light")
    rep["verify_equal"] = list(a) == list(b)
    rep["verify_valid"] = sum(1 for r in a if r["valid"])
    W.barrier()
    with open(out_path, "w") as f:
        json.dump(rep, f)
    dev.close()
    W.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
