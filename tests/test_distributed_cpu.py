"""Multi-process (gloo, world_size 2 and 4, CPU) rehearsal of the RCCL paths in parallel/ and the
miner: work-packet broadcast, max/sum reductions, in-place DAG shard all-gather (slices filled
with golden ethash items), the mining loop's record all-gather (miner/service.Comm), and the
disjoint nonce partition bench.py and the miner use. Same code as the GPU path, gloo backend.
World size 1 with forced collectives is the one-rank process group a 1-GPU box runs over RCCL."""
import os
import socket
import struct
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        import torch

        from nodexa_chain_core_amd import _core
        from nodexa_chain_core_amd.parallel import dag as pdag
        from nodexa_chain_core_amd.parallel import world as W
        from nodexa_chain_core_amd.miner.search import SlotResult
        from nodexa_chain_core_amd.miner.service import Comm, pack_record, unpack_record
        from nodexa_chain_core_amd.ops.kawpow import Share

        w = W.init(use_gpu=False, force_collectives=world == 1)
        assert w.backend == "gloo" and w.world_size == world and w.collective
        # 1. work packet broadcast from rank 0
        pkt = struct.pack("<32sQII", bytes(range(32)), 7, 1234, 0)
        got = W.broadcast_bytes(pkt if rank == 0 else None, len(pkt))
        assert got == pkt
        # 2. reductions
        assert W.all_reduce_max(float(rank) + 0.5) == world - 0.5
        assert W.all_reduce_sum_int(rank + 1) == world * (world + 1) // 2
        # 2b. resident batch verify below the shard threshold: rank 0's verdict broadcast to all
        from nodexa_chain_core_amd.models.verify import _broadcast_verdict

        v0 = {"accepted": 9990, "reject": {"index": 9990, "reason": "high-hash"}, "dos": 50}
        got = _broadcast_verdict(w, v0 if rank == 0 else None)
        assert got["accepted"] == 9990 and got["reject"] == {"index": 9990, "reason": "high-hash"} and got["dos"] == 50
        got = _broadcast_verdict(w, {"accepted": 10000, "reject": None, "dos": 0} if rank == 0 else None)
        assert got["accepted"] == 10000 and got["reject"] is None
        try:  # a failure on rank 0 reaches every rank instead of leaving them in the broadcast
            _broadcast_verdict(w, ValueError("device lost") if rank == 0 else None)
            raise AssertionError("no exception")
        except (ValueError, RuntimeError) as e:
            assert "device lost" in str(e)
        # 3. DAG shard all-gather: each rank fills its slice with golden 2048-bit items
        ctx = _core.get_epoch_context(0)
        per_items = 8
        full = torch.zeros(world * per_items * 256, dtype=torch.uint8)
        for i in range(per_items):
            item = rank * per_items + i
            full[(item * 256):(item + 1) * 256] = torch.frombuffer(bytearray(_core.dataset_item_2048(ctx, item)),
                                                                   dtype=torch.uint8)
        pdag.allgather_shards(full, per_items * 256)
        raw = full.numpy().tobytes()
        for item in range(world * per_items):
            assert raw[item * 256:(item + 1) * 256] == _core.dataset_item_2048(ctx, item), item
        # 4. the mining loop's record all-gather: rank r reports r+1 shares with nonces r*1000+i
        comm = Comm(60.0)
        shares = [Share(rank * 1000 + i, bytes([rank]) * 32, bytes([i]) * 32) for i in range(rank + 1)]
        recs = [unpack_record(x) for x in comm.all_gather(pack_record(SlotResult(7, 0, 64, 64 + rank, shares)))]
        assert [s.nonce for r in recs for s in r.shares] == [r * 1000 + i for r in range(world) for i in range(r + 1)]
        assert comm.all_reduce_sum([rank + 1, 1]) == [world * (world + 1) // 2, world]
        assert comm.broadcast(b"w" * 144 if rank == 0 else None, 144) == b"w" * 144
        # 5. nonce partition of bench.py: disjoint windows across ranks and steps
        batch, base = 1 << 20, 0x5EED_0000_0000_0000
        windows = [(base + (i * world + r) * batch, batch) for i in range(3) for r in range(world)]
        ends = sorted(windows)
        assert all(a[0] + a[1] <= b[0] for a, b in zip(ends, ends[1:]))
        W.barrier()
        W.shutdown()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, traceback.format_exc() or repr(e)))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_gloo_collectives(world):
    """World 8 = one rank per GPU of an MI355X node: 8-shard DAG gather, record gather of 8 ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=280) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert results == {r: "ok" for r in range(world)}, results


def _verify_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        from nodexa_chain_core_amd import _core
        from nodexa_chain_core_amd.models import synthetic
        from nodexa_chain_core_amd.parallel import world as W
        from nodexa_chain_core_amd.parallel.verify import verify_headers_distributed

        W.init(use_gpu=False)
        params, headers = synthetic.load(os.path.join(ROOT, "tests", "data", "testnet_kawpow_10k.hdr"))
        act = params.kawpow_activation_time
        batch = [_core.BlockHeader.deserialize(h.serialize(act), act) for h in headers[:37]]
        batch[20].mix_hash = bytes(32)  # one invalid header, owned by whichever rank gets slot 20
        res = verify_headers_distributed(params, batch)
        q.put((rank, [(r["valid"], r.get("reason"), r["hash"]) for r in res]))
        W.barrier()
        W.shutdown()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, traceback.format_exc() or repr(e)))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_distributed_verify_matches_single_process(world):
    """parallel/verify.py: full-hash work split over ranks + all_gather_into_tensor gives every
    rank the single-process verify_headers result (uneven split included: 37 headers)."""
    from nodexa_chain_core_amd import _core
    from nodexa_chain_core_amd.models import synthetic
    from nodexa_chain_core_amd.models.verify import verify_headers

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_verify_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=280) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    params, headers = synthetic.load(os.path.join(ROOT, "tests", "data", "testnet_kawpow_10k.hdr"))
    act = params.kawpow_activation_time
    batch = [_core.BlockHeader.deserialize(h.serialize(act), act) for h in headers[:37]]
    batch[20].mix_hash = bytes(32)
    want = [(r["valid"], r.get("reason"), r["hash"]) for r in verify_headers(params, batch, threads=4)]
    assert not want[20][0] and all(v for v, _, _ in want[:20])
    for r in range(world):
        assert results[r] == want, results[r] if isinstance(results[r], str) else r


def _elastic_worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        import torch

        from nodexa_chain_core_amd.parallel import dag as pdag
        from nodexa_chain_core_amd.parallel import world as W

        W.init(use_gpu=False)
        assert W.all_reduce_sum_int(1) == world
        if rank == world - 1:  # this rank "dies": it leaves without another collective
            q.put((rank, "left"))
            return
        w = W.shrink(list(range(world - 1)))
        assert w.world_size == world - 1 and w.rank == rank
        assert W.all_reduce_sum_int(rank + 1) == (world - 1) * world // 2
        pkt = bytes(range(96))
        assert W.broadcast_bytes(pkt if w.rank == 0 else None, 96) == pkt
        per = 16
        full = torch.zeros(w.world_size * per, dtype=torch.uint8)
        full[w.rank * per:(w.rank + 1) * per] = w.rank + 1
        pdag.allgather_shards(full, per)
        assert full.tolist() == [r + 1 for r in range(w.world_size) for _ in range(per)]
        # the nonce partition re-derives from the new (rank, world_size): disjoint, gap-free
        batch, base = 1 << 10, 7 << 40
        mine = [(base + (i * w.world_size + w.rank) * batch) for i in range(3)]
        q.put((rank, mine))
        W.barrier()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, traceback.format_exc() or repr(e)))


@pytest.mark.timeout(300)
def test_elastic_shrink_after_rank_loss():
    """parallel/world.shrink: after rank 2 of 3 is lost the survivors rebuild the communicator
    (new_group with local synchronisation) and every collective and the nonce partition carry on
    over 2 ranks (SURVEY §5 elastic world size)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_elastic_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=280) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert results[2] == "left", results
    starts = sorted(results[0] + results[1])
    assert all(isinstance(results[r], list) for r in (0, 1)), results
    assert [b - a for a, b in zip(starts, starts[1:])] == [1 << 10] * 5
