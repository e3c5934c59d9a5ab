"""Process-group bring-up: one process per GPU, torch.distributed over RCCL.

On ROCm the "nccl" backend *is* RCCL; on the 8 MI355X of a node its
collectives run over the point-to-point xGMI mesh (7 links per GPU). CPU-only
runs (tests, rehearsals) use "gloo" with the same code paths.

Rendezvous always uses 127.0.0.1 (the container hostname may not resolve).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class World:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    group: object = None            # process group of the collectives (None = the default group)
    ranks: tuple[int, ...] = ()     # global ranks of the group members, index = rank in the group

    def global_rank(self, r: int) -> int:
        return self.ranks[r] if self.ranks else r

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def collective(self) -> bool:
        """There is a process group: collectives run (also at world size 1 when forced)."""
        return self.backend != "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_WORLD: World | None = None
_INIT_GROUP = None  # the collective-timeout group init() made (None: the default group)


def is_init_group(group) -> bool:
    """`group` is the whole-world collective group of init(), shared by this module's helpers
    (users that must abort their communicator alone, miner/service.Comm, make their own)."""
    return group is None or group is _INIT_GROUP


def rendezvous_timeout() -> int:
    """Timeout of the default group (NODEXA_RENDEZVOUS_TIMEOUT, default 300 s): the start-up
    rendezvous and full-mesh connect, which must tolerate ranks that start seconds apart (a loaded
    host, a cold torch import). On RCCL failure detection does not use it: the mining loop's
    collectives run on a group of their own with the collective timeout (miner/service.Comm), and
    this module's helpers on the group init(collective_timeout_s=...) makes."""
    return int(os.environ.get("NODEXA_RENDEZVOUS_TIMEOUT", "300"))


def init(use_gpu: bool | None = None, timeout_s: int = 600, device_index: int | None = None,
         rank: int | None = None, world_size: int | None = None, elastic: bool = False,
         force_collectives: bool | None = None, collective_timeout_s: float | None = None) -> World:
    """Initialise from RANK/WORLD_SIZE/LOCAL_RANK (torchrun, or the node's spawned miner ranks)
    or single-process; `rank` / `world_size` override the environment. `device_index`: the GPU
    of this rank (default: LOCAL_RANK). `force_collectives` (env NODEXA_FORCE_COLLECTIVES=1):
    make a process group even for one rank, so every collective of the miner, the DAG build and
    batch verify really runs (one-rank RCCL on a 1-GPU box exercises the 8-GPU code path).

    `timeout_s` bounds the start-up rendezvous (callers pass rendezvous_timeout(), minutes). With
    `collective_timeout_s` below it, the collectives of this module (barrier, all_reduce_*, the
    sharded DAG gather of parallel/dag.py, batch verify) run on a group of their own created with
    that shorter timeout, so a rank lost mid-collective is detected in collective time, not
    rendezvous time. RCCL only: a gloo group connects its full mesh under its own timeout, and
    host rehearsals whose ranks start seconds apart keep the default group."""
    global _WORLD
    rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
    world_size = int(os.environ.get("WORLD_SIZE", "1")) if world_size is None else int(world_size)
    if force_collectives is None:
        force_collectives = os.environ.get("NODEXA_FORCE_COLLECTIVES", "0") == "1"
    if _WORLD is not None:
        # a single-process world left by an earlier user of this process (no communicator to
        # tear down) gives way to a request for a real one; anything else is reused as it is
        if not ((world_size > 1 or force_collectives) and not _WORLD.collective and not dist.is_initialized()):
            return _WORLD
        _WORLD = None
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(device_index if device_index is not None
                              else local_rank % max(1, torch.cuda.device_count()))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    backend = "none"
    if world_size > 1 or force_collectives:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        backend = "nccl" if use_gpu else "gloo"
        # NODEXA_DIST_BACKEND=gloo: ranks that share one GPU (a multi-rank rehearsal on a 1-GPU box:
        # RCCL refuses two ranks on one device) exchange through gloo instead
        backend = os.environ.get("NODEXA_DIST_BACKEND", backend)
        if elastic and use_gpu:
            # a collective that times out must raise to the caller (which aborts the communicator
            # and re-forms the group over the survivors), not make RCCL's watchdog end the process
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
        if backend == "nccl":
            # RCCL's internal streams at high priority: with 4 hardware queues per process, a
            # normal-priority stream can share a queue with the search stream, and a collective
            # queued there waits behind the ~117 ms search window already queued (profiles r4b)
            os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
        kw = {}
        if use_gpu:
            kw["device_id"] = device
        dist.init_process_group(backend=backend, rank=rank, world_size=world_size,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    global _INIT_GROUP
    group = None
    if backend == "nccl" and collective_timeout_s is not None and collective_timeout_s < timeout_s:
        group = dist.new_group(ranks=list(range(world_size)),
                               timeout=datetime.timedelta(seconds=float(collective_timeout_s)))
    _INIT_GROUP = group
    _WORLD = World(rank, world_size, local_rank, backend, device, group, tuple(range(world_size)))
    return _WORLD


def shrink(survivors: list[int], timeout_s: int = 120) -> World:
    """Elastic world size: rebuild the communicator over the surviving ranks after a
    rank is lost, and make it the group every collective here uses. Only the survivors call
    this (local synchronisation: a dead rank never joins). Ranks are renumbered 0..n-1 in the
    order of `survivors`' global ranks, so the nonce partition (rank, world_size) and shard
    ownership simply re-derive from the new World."""
    global _WORLD
    w = get()
    members = sorted(set(int(r) for r in survivors))
    g = w.global_rank(w.rank)
    if g not in members:
        raise RuntimeError(f"rank {g} is not among the survivors {members}")
    if len(members) == len(w.ranks or range(w.world_size)):
        return w
    grp = dist.new_group(ranks=members, timeout=datetime.timedelta(seconds=timeout_s),
                         use_local_synchronization=True)
    _WORLD = World(members.index(g), len(members), w.local_rank, w.backend, w.device, grp, tuple(members))
    return _WORLD


def get() -> World:
    return _WORLD if _WORLD is not None else init()


def shutdown() -> None:
    global _WORLD, _INIT_GROUP
    if _WORLD is not None and _WORLD.collective and dist.is_initialized():
        dist.destroy_process_group()
    _WORLD = None
    _INIT_GROUP = None


def barrier() -> None:
    w = get()
    if w.collective:
        if w.backend == "nccl":
            dist.barrier(group=w.group, device_ids=[w.device.index])
        else:
            dist.barrier(group=w.group)


def broadcast_bytes(payload: bytes | None, size: int, src: int = 0) -> bytes:
    """Broadcast a fixed-size packet (e.g. the 96-byte work packet) from `src`: a device tensor
    over RCCL, a host tensor over gloo (which would copy a device tensor through the host anyway)."""
    w = get()
    t = torch.zeros(size, dtype=torch.uint8, device=w.device if w.backend == "nccl" else "cpu")
    if w.rank == src and payload is not None:
        if len(payload) != size:
            raise ValueError("payload size mismatch")
        t.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
    if w.collective:
        dist.broadcast(t, src=w.global_rank(src), group=w.group)
    return bytes(t.cpu().numpy().tobytes())


def all_reduce_max(x: float) -> float:
    w = get()
    if not w.collective:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=w.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=w.group)
    return float(t.item())


def all_reduce_sum_int(x: int) -> int:
    w = get()
    if not w.collective:
        return x
    t = torch.tensor([x], dtype=torch.int64, device=w.device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=w.group)
    return int(t.item())
