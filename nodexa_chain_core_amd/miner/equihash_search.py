"""Equihash(200,9) windows for the mining loop (miner/search.py two-slot protocol).

The chain's Equihash extension (csrc/chain/primitives.hpp) hashes
I = 80-byte header prefix || nonce256, and a block is valid when one of I's solutions makes
SHA256d(serialized header) <= nBits target. A window of `count` nonces is `count` solver
instances: nonce k of the window stands for nonce256 = le64(start + k) || 0^24, so the ranks'
64-bit nonce partition (rank << 56) carries over unchanged.

* `EquihashGpuDevice`: one `ops.equihash.EquihashSolver` with `num_inst` instances per launch
  (16: ~8.4 ms of device work, so the loop's per-step host work and collectives hide behind the
  window that is running); the solver keeps two launches in flight on its stream with two pinned
  landing buffers, one per slot. Every solution is verified on the device (eq_verify_slots)
  before it is counted; the host only SHA256d's the candidate headers.
* `EquihashCpuDevice`: the C++ golden solver (~2.3 s per nonce on one core) for CPU-only nodes and
  the gloo rehearsals of the loop.

`hashes` of an Equihash SlotResult is the number of distinct valid solutions found (the Sol/s of
the bench); shares are the solutions whose block hash meets the work's boundary (at most
MAX_EQ_SHARES per window, the rest are counted but not shipped: one block per job is enough).
"""
from __future__ import annotations

import time

from .. import core
from .search import ALGO_EQUIHASH, EquihashShare, SlotResult, Work, equihash_block_hash, equihash_nonce256

_core = core()
MAX_EQ_SHARES = 4
PARAMS = _core.EquihashParams(200, 9)


def _passing(work: Work, start: int, per_nonce: list[list[bytes]]) -> tuple[list[EquihashShare], int]:
    """Shares of a window: every (nonce, packed solution) whose SHA256d header hash <= boundary."""
    target = work.target()
    shares, sols = [], 0
    for k, packed in enumerate(per_nonce):
        sols += len(packed)
        for sol in packed:
            bh = equihash_block_hash(work.header, start + k, sol)
            if int.from_bytes(bh, "little") <= target and len(shares) < MAX_EQ_SHARES:
                shares.append(EquihashShare(start + k, sol, bh))
    return shares, sols


class EquihashGpuDevice:
    name = "gpu-equihash"
    algo = ALGO_EQUIHASH

    def __init__(self, device: int = 0, num_inst: int = 16):
        import os

        import torch

        from ..ops.equihash import EquihashSolver

        self.torch = torch
        self.device = int(device)
        self.num_inst = int(num_inst)
        # one solver on one stream serves both slots (the solver keeps two launches in flight); a
        # solver + stream per slot measured no gain (profiles/README r4g: 7.5-8.3 vs 8.0-8.1 ms per
        # window; r4z: the two streams landed on one hardware queue, +1 ms per step) and was removed
        with torch.cuda.device(self.device):
            self.streams = [torch.cuda.Stream(device=self.device)] * 2
            with torch.cuda.stream(self.streams[0]):
                self.solvers = [EquihashSolver(num_inst=self.num_inst, device=self.device)] * 2
            self.starts = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            self.ends = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        self.stream = self.streams[0]
        self.solver = self.solvers[0]
        self.meta: list[tuple | None] = [None, None]
        self.order: list[int] = []  # slots in launch order (collected oldest first)

    def window_for(self, work: Work, window: int) -> int:
        return self.num_inst

    def submit(self, slot: int, work: Work, start: int, count: int) -> None:
        torch = self.torch
        inputs = [work.header + equihash_nonce256(start + k) for k in range(self.num_inst)]
        st = self.streams[slot]
        with torch.cuda.device(self.device), torch.cuda.stream(st):
            self.starts[slot].record(st)
            self.solvers[slot].launch(inputs)
            self.ends[slot].record(st)
        self.meta[slot] = (work, start)
        self.order.append(slot)

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        from ..ops.equihash import pack_solutions
        from .search import DeviceHung

        if not self.order or self.order[0] != slot:
            raise RuntimeError("Equihash slots must be collected in launch order")
        ev = self.ends[slot]
        if timeout_s is not None:
            deadline = time.monotonic() + timeout_s
            while not ev.query():
                if time.monotonic() > deadline:
                    raise DeviceHung(f"gpu{self.device}: Equihash window did not finish in {timeout_s:.0f}s")
                time.sleep(0.0002)
        self.order.pop(0)
        arrays = self.solvers[slot].collect_arrays(verify="device")
        work, start = self.meta[slot]
        self.meta[slot] = None
        shares, sols = _passing(work, start, [pack_solutions(a) if len(a) else [] for a in arrays])
        return SlotResult(work.job_id, start, self.num_inst, sols, shares, self.starts[slot].elapsed_time(ev), 0,
                          ALGO_EQUIHASH)

    def abort(self) -> None:
        """Queued Equihash launches are short (~9 ms) and carry no stale check: they finish and the
        leader drops their shares as stale."""

    def synchronize(self) -> None:
        for st in self.streams:
            st.synchronize()

    def close(self) -> None:
        pass


class EquihashCpuDevice:
    """The host golden solver, `count` nonces per window (1 by default)."""

    name = "cpu-equihash"
    algo = ALGO_EQUIHASH
    device = -1

    def __init__(self, window: int = 1):
        self.window = max(1, int(window))
        self.meta: list[tuple | None] = [None, None]
        self.generation = 0

    def window_for(self, work: Work, window: int) -> int:
        return self.window

    def submit(self, slot: int, work: Work, start: int, count: int) -> None:
        self.meta[slot] = (work, start, min(count, self.window), self.generation)

    def wait(self, slot: int, timeout_s: float | None = None) -> SlotResult:
        work, start, count, gen = self.meta[slot]
        self.meta[slot] = None
        if gen != self.generation:
            return SlotResult(work.job_id, start, count, 0, [], 0.0, 1, ALGO_EQUIHASH)
        t0 = time.perf_counter()
        per = []
        for k in range(count):
            sols, _ = _core.equihash_solve_cpu(PARAMS, work.header + equihash_nonce256(start + k), 16, 0)
            uniq = {tuple(s) for s in sols}
            per.append([_core.equihash_pack(PARAMS, list(s)) for s in sorted(uniq)])
        shares, n = _passing(work, start, per)
        return SlotResult(work.job_id, start, count, n, shares, (time.perf_counter() - t0) * 1e3, 0, ALGO_EQUIHASH)

    def abort(self) -> None:
        self.generation += 1

    def synchronize(self) -> None:
        pass

    def close(self) -> None:
        pass
