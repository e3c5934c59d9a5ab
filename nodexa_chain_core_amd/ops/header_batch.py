"""Device-resident batch header verification (BASELINE config 5).

Reference: ProcessNewBlockHeaders (src/validation.cpp:12017-12035) runs CheckBlockHeader
(:11638-11665: full KawPow light-mode hash + mix_hash equality) and ContextualCheckBlockHeader
(:11811-11875: DarkGravityWave nBits, MTP, future time, version) header by header under cs_main.

Here the batch (csrc/chain/headerbatch.hpp: parsed once from its wire bytes, packed into 128-byte
rows in one parallel pass) crosses the PCIe bus twice in total:

  host  -> device  one copy: rows | kinds | DGW ancestor series | Equihash messages, solutions
                   and serialized headers (one pinned staging buffer)
  device           kawpow_mixonly_batch (SHA256d header hash + mix-only final + nBits boundary),
                   hb_jobs, kawpow_verify_waves per epoch range (resident DAG, per-epoch program
                   table resident too; the ranges side by side on their own streams), hb_verdict;
                   beside that chain eq_verify + sha256d_batch and dgw_batch on a side stream;
                   then hb_eq_scatter — ordered by events, no host synchronisation in between
  device -> host   one copy: per-header code | block hash | expected nBits

and the host keeps only the serial index insert (HeaderChain.accept_batch, native, GIL released,
with the device's block hashes and nBits). Over N ranks each GPU runs the rows of its slice and the
compact results are all-gathered device to device (RCCL) before the single copy back.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .. import core
from . import runtime

_core = core()
ROW = 128
CODES = {1: "invalid-mix-hash", 2: "high-hash", 3: "invalid-solution"}
_ALIGN = 256
# full hashes with wave-uniform programs (kawpow_verify_waves: program in SGPRs, mix in VGPRs);
# test hook only: False runs the LDS-mix interpreter (kawpow_verify_dag), the bit-exactness oracle
# of tests/test_gpu_resident_verify.py
WAVES = True


def _al(x: int) -> int:
    return (x + _ALIGN - 1) // _ALIGN * _ALIGN


class ResidentHeaderVerifier:
    """One device's pipeline: persistent device / pinned buffers (grown on demand), a stream,
    resident per-epoch ProgPoW program tables; DAGs come from ops/verify's resident-epoch LRU."""

    def __init__(self, device: int = 0):
        runtime.require_gpu()
        self.device = int(device)
        self.h = runtime.hip()
        self.dev = torch.device("cuda", self.device)
        with torch.cuda.device(self.dev):
            self.stream = torch.cuda.Stream(device=self.dev)
            self.side = [torch.cuda.Stream(device=self.dev) for _ in range(3)]  # Equihash + DGW, epoch ranges
            # raw HIP events, recorded / waited through the runtime's one-call helpers (torch's
            # Python wrappers cost several microseconds per operation on this issue path)
            h = self.h
            self.ev_start, self.ev_end = h.event_create(True), h.event_create(True)
            self.ev_in, self.ev_jobs = h.event_create(), h.event_create()
            self.ev_side = [h.event_create() for _ in self.side]
            # the early copy of block hashes + nBits (models/verify.py prepares the index insert
            # from it while the full hashes run), made at the end of the side stream
            self.ev_early = h.event_create()
            self.ev_dgw = h.event_create()
        self.cap = 0
        self.in_cap = 0
        self.programs: dict[int, torch.Tensor] = {}
        self.k = {name: runtime.static_kernel("header_batch", name) for name in ("hb_jobs", "hb_verdict", "hb_eq_scatter")}
        self.k_mo = runtime.static_kernel("sha256d", "kawpow_mixonly_batch")
        self.k_sha = runtime.static_kernel("sha256d", "sha256d_batch")
        self.k_dag = runtime.static_kernel("kawpow_verify_light", "kawpow_verify_dag")
        self.k_waves = runtime.static_kernel("kawpow_verify_light", "kawpow_verify_waves")
        self.k_eq = runtime.static_kernel("equihash", "eq_verify")
        self.k_dgw = runtime.static_kernel("dgw", "dgw_batch")
        from .equihash import blake2b_h0

        self.h0 = blake2b_h0()

    # ------------------------------------------------------------------ resident state
    def program_table(self, epoch: int) -> torch.Tensor:
        """The epoch's 2500 ProgPoW programs (64 words each), resident (per-epoch setup)."""
        t = self.programs.get(epoch)
        if t is None:
            per = _core.EPOCH_LENGTH // 3
            raw = _core.kawpow_programs_bytes(list(range(epoch * per, (epoch + 1) * per)))
            with torch.cuda.device(self.dev):
                t = torch.frombuffer(bytearray(raw), dtype=torch.int32).to(self.dev)
            if len(self.programs) >= 8:
                self.programs.pop(next(iter(self.programs)))
            self.programs[epoch] = t
        return t

    def _ensure(self, n: int, in_bytes: int) -> None:
        with torch.cuda.device(self.dev):
            if n > self.cap:
                cap = max(n, 2 * self.cap, 1024)
                self.mo = torch.empty(cap * 128, dtype=torch.uint8, device=self.dev)
                self.jobs = torch.empty(cap * 48, dtype=torch.uint8, device=self.dev)
                self.jprog = torch.empty(cap, dtype=torch.int32, device=self.dev)
                self.full = torch.empty(cap * 16, dtype=torch.int32, device=self.dev)
                self.out = torch.empty(cap * 37, dtype=torch.uint8, device=self.dev)  # codes | hashes | bits
                self.gath = torch.empty(cap * 33 * 2 + 64 * 33, dtype=torch.uint8, device=self.dev)
                self.out_host = torch.empty(cap * 37, dtype=torch.uint8).pin_memory()
                self.early_host = torch.empty(cap * 36, dtype=torch.uint8).pin_memory()  # hashes | bits
                self.cap = cap
            if in_bytes > self.in_cap:
                cap = max(in_bytes, 2 * self.in_cap)
                self.din = torch.empty(cap, dtype=torch.uint8, device=self.dev)
                self.in_host = torch.empty(cap, dtype=torch.uint8).pin_memory()
                self.in_cap = cap

    # ------------------------------------------------------------------ one batch
    def plan(self, batch) -> dict | None:
        """Host-side numpy planning (no device work): epoch ranges of the KawPow rows. None when
        the batch is not in height order (the resident path wants contiguous epoch ranges)."""
        n = len(batch)
        got = batch.kawpow_plan(_core.EPOCH_LENGTH)  # one native pass over the rows
        if got is None:
            return None
        ranges, heights, times, bits = got
        return {"rows": np.frombuffer(batch.rows, dtype=np.uint8).reshape(n, ROW),
                "kinds": np.frombuffer(batch.kinds, dtype=np.uint8), "ranges": ranges,
                "heights": np.frombuffer(heights, dtype="<u4"), "times": np.frombuffer(times, dtype="<u4"),
                "bits": np.frombuffer(bits, dtype="<u4")}

    @staticmethod
    def wave_slots(rows_idx: np.ndarray, heights: np.ndarray, lo: int) -> np.ndarray:
        """kawpow_verify_waves' slot table for the KawPow rows `rows_idx` of one epoch range: the
        rows grouped by ProgPoW period (height // 3), each period's rows in slots of 4 (one wave64
        of four 16-lane groups per 4 rows, -1 for an idle group), values relative to `lo`."""
        if len(rows_idx) == 0:
            return np.zeros(0, dtype=np.int32)
        per = heights[rows_idx] // 3
        order = np.argsort(per, kind="stable")
        r, per = rows_idx[order], per[order]
        start = np.flatnonzero(np.r_[True, per[1:] != per[:-1]])  # first row of each period run
        length = np.diff(np.r_[start, len(per)])
        waves = (length + 3) // 4
        base = np.r_[0, np.cumsum(waves)[:-1]] * 4  # first slot of each run
        pos = np.arange(len(per)) - np.repeat(start, length)
        slots = np.full(int(waves.sum()) * 4, -1, dtype=np.int32)
        slots[np.repeat(base, length) + pos] = (r - lo).astype(np.int32)
        return slots

    def run(self, params, batch, series, plan: dict | None = None, world=None, overlap=None) -> dict:
        """Verify the PoW of every header and compute every header's DGW nBits on the device.
        `series`: (ancestor times bytes, ancestor bits bytes, a, base_height) of the batch's parent
        (HeaderChain.dgw_ancestors) or None. `overlap(early)`: host work to run while the device
        works (models/verify.py: the batch's deferred header decode, then the index insert's
        prepare phase); `early()` waits for the block hashes + DGW nBits only (one rank: they are
        complete before the full hashes are) and returns them as (n, 32) u8 / (n,) u32 views, or
        None on a multi-rank world. Returns codes (n,) u8, hashes (n, 32) u8, bits (n,) u32 as
        numpy views of the pinned result buffer, plus timings."""
        from . import verify as V

        t0 = time.perf_counter()
        n = len(batch)
        plan = plan or self.plan(batch)
        if plan is None:
            raise ValueError("batch is not in height order")
        rows, kinds = plan["rows"], plan["kinds"]
        ws, rank = (world.world_size, world.rank) if world is not None and world.collective else (1, 0)
        per = -(-n // ws)
        lo_r, hi_r = min(n, rank * per), min(n, (rank + 1) * per)
        eq_index = np.frombuffer(batch.eq_index, dtype=np.uint32)
        mine_eq = np.flatnonzero((eq_index >= lo_r) & (eq_index < hi_r))
        m = len(mine_eq)
        eq_len = int(batch.eq_ser_len)
        if m and not batch.eq_uniform:
            raise ValueError("malformed Equihash header in the batch")  # process_batch_resident filters these
        # staging layout (one pinned buffer, one H2D copy)
        a = series[2] if series is not None else 0
        off = {}
        cur = 0
        # per epoch range of this rank: the wave-uniform slot table (kawpow_verify_waves)
        slot_tabs = []  # int32 bytes per range
        if WAVES:
            for epoch, lo, hi in plan["ranges"]:
                lo, hi = max(lo, lo_r), min(hi, hi_r)
                if lo < hi:
                    slot_tabs.append(_core.wave_slots(kinds, plan["heights"], lo, hi))
        slot_lens = [len(t) // 4 for t in slot_tabs]
        nslots = sum(slot_lens)
        for name, size in (("rows", n * ROW), ("kinds", n), ("times", (a + n) * 4), ("bits", (a + n) * 4),
                           ("eq_index", m * 4), ("eq_msgs", m * 128), ("eq_sols", m * 1344),
                           ("eq_ser", m * eq_len), ("eq_verdict", m * 4), ("eq_hash", m * 32),
                           ("slots", nslots * 4)):
            off[name] = (cur, size)
            cur = _al(cur + size)
        self._ensure(n, cur)
        stage = self.in_host.numpy()

        # the whole upload staged by one native call: (offset, bytes-like) parts, bounds checked
        parts = [(off["rows"][0], batch.rows), (off["kinds"][0], batch.kinds)]
        if series is not None:  # the ancestors' (nTime, nBits), then the batch's own
            parts += [(off["times"][0], series[0]), (off["times"][0] + 4 * a, plan["times"]),
                      (off["bits"][0], series[1]), (off["bits"][0] + 4 * a, plan["bits"])]
        o = off["slots"][0]
        for t, ln in zip(slot_tabs, slot_lens):
            parts.append((o, t))
            o += 4 * ln
        if m == len(eq_index):  # every Equihash header is this rank's: the packed arrays as they are
            parts += [(off["eq_index"][0], batch.eq_index), (off["eq_msgs"][0], batch.eq_msgs),
                      (off["eq_sols"][0], batch.eq_sols), (off["eq_ser"][0], batch.eq_ser)]
        elif m:
            parts += [(off["eq_index"][0], eq_index[mine_eq].astype(np.uint32)),
                      (off["eq_msgs"][0], np.ascontiguousarray(np.frombuffer(batch.eq_msgs, np.uint8).reshape(-1, 128)[mine_eq])),
                      (off["eq_sols"][0], np.ascontiguousarray(np.frombuffer(batch.eq_sols, np.uint8).reshape(-1, 1344)[mine_eq])),
                      (off["eq_ser"][0], np.ascontiguousarray(np.frombuffer(batch.eq_ser, np.uint8).reshape(-1, eq_len)[mine_eq]))]
        _core.copy_into_many(stage, parts)
        t_pack = time.perf_counter()
        h = self.h
        base = self.din.data_ptr()
        P = lambda name: base + off[name][0]  # noqa: E731
        out = self.out.data_ptr()
        lim = bytes(params.pow_limit)
        cp = int(params.last_checkpoint_height)
        nr = hi_r - lo_r

        def glue(which: int, first: int, count: int, st: int) -> None:
            kern = self.k[("hb_jobs", "hb_verdict", "hb_eq_scatter")[which]]
            h.launch_header_batch(kern, which, P("rows"), P("kinds"), self.mo.data_ptr(), self.jobs.data_ptr(),
                                  self.jprog.data_ptr(), self.full.data_ptr(), out, P("eq_index"), P("eq_verdict"),
                                  P("eq_hash"), n, m, first, count, _core.EPOCH_LENGTH, cp, lim, st)

        # every epoch DAG of the plan resolved (built or pinned in the LRU) before the first launch:
        # a build inside the issue loop could evict a DAG a side-stream range is still reading
        epochs_dev = {}
        V.prefetch_contexts({e for e, lo, hi in plan["ranges"] if max(lo, lo_r) < min(hi, hi_r)}, self.device)
        for epoch, lo, hi in plan["ranges"]:
            if max(lo, lo_r) < min(hi, hi_r) and epoch not in epochs_dev:
                epochs_dev[epoch] = V._device_epoch(epoch, self.device)
        if len(epochs_dev) > V.MAX_RESIDENT_DAGS:
            raise ValueError("batch spans more epochs than the resident DAGs")
        main = self.stream
        with torch.cuda.device(self.dev), torch.cuda.stream(main):
            s = int(main.cuda_stream)
            h.event_record(self.ev_start, s)
            h.memcpy_async(base, self.in_host.data_ptr(), cur, s, "htod")
            if series is None:
                h.memset_async(out + n * 33, 0, n * 4, s)  # nBits 0 = the host decides
            h.event_record(self.ev_in, s)
            # Equihash solutions + block hashes and the DGW nBits depend only on the upload: a side
            # stream runs them beside the KawPow chain (mix-only -> jobs -> full hashes -> verdicts)
            s0 = int(self.side[0].cuda_stream)
            h.stream_wait_event(s0, self.ev_in)
            if series is not None:
                # DGW (~120 us, latency-bound per lane) on a stream of its own, beside the Equihash
                # work: the early copy below needs both
                sd = int(self.side[-1].cuda_stream)
                h.stream_wait_event(sd, self.ev_in)
                c = _core.dgw_constants(params)
                h.launch_dgw(self.k_dgw, P("times"), P("bits"), out + n * 33, a, n, series[3], c["dgw_activation_block"],
                             c["kawpow_time"], c["equihash_time"], c["limits"], c["compacts"], c["target_timespan"], sd)
                h.event_record(self.ev_dgw, sd)
            if m:
                h.launch_equihash_verify(self.k_eq, self.h0, P("eq_msgs"), 112, m, P("eq_sols"), P("eq_verdict"), s0)
                h.launch_sha256d(self.k_sha, P("eq_ser"), eq_len, eq_len, m, P("eq_hash"), False, s0)
            if m:
                glue(2, 0, 0, s0)  # Equihash codes + block hashes (hb_verdict leaves those rows alone)
            if series is not None:
                h.stream_wait_event(s0, self.ev_dgw)  # ev_side[0]: the Equihash work and DGW done
            h.event_record(self.ev_side[0], s0)
            if nr:
                h.launch_kawpow_mixonly(self.k_mo, P("rows") + lo_r * ROW, nr, ROW, self.mo.data_ptr() + lo_r * 128, s)
                glue(0, lo_r, nr, s)  # jobs + the KawPow block hashes
            h.event_record(self.ev_jobs, s)
            if nr:
                # one full-hash launch per epoch range, the ranges side by side: each is bound by
                # its 64 dependent rounds per job, not by width
                slot_off = [sum(slot_lens[:j]) for j in range(len(slot_lens))]  # in slots
                k = 0
                for epoch, lo, hi in plan["ranges"]:
                    lo, hi = max(lo, lo_r), min(hi, hi_r)
                    if lo >= hi:
                        continue
                    st = main if k == 0 else self.side[1 + (k - 1) % (len(self.side) - 1)]
                    if st is not main:
                        h.stream_wait_event(int(st.cuda_stream), self.ev_jobs)
                    ep = epochs_dev[epoch]
                    if WAVES:
                        h.launch_kawpow_verify_waves(self.k_waves, ep.dag.data_ptr(), ep.items2048, ep.l1.data_ptr(),
                                                     self.jobs.data_ptr() + lo * 48,
                                                     self.program_table(epoch).data_ptr(), _core.EPOCH_LENGTH // 3,
                                                     self.jprog.data_ptr() + lo * 4, hi - lo,
                                                     P("slots") + slot_off[k] * 4, slot_lens[k],
                                                     self.full.data_ptr() + lo * 64, int(st.cuda_stream))
                    else:
                        h.launch_kawpow_verify_dag(self.k_dag, ep.dag.data_ptr(), ep.items2048, ep.l1.data_ptr(),
                                                   self.jobs.data_ptr() + lo * 48, self.program_table(epoch).data_ptr(),
                                                   _core.EPOCH_LENGTH // 3, self.jprog.data_ptr() + lo * 4, hi - lo,
                                                   self.full.data_ptr() + lo * 64, int(st.cuda_stream))
                    if st is not main:
                        ev = self.ev_side[1 + (k - 1) % (len(self.side) - 1)]
                        h.event_record(ev, int(st.cuda_stream))
                        h.stream_wait_event(s, ev)
                    k += 1
                glue(1, lo_r, nr, s)
            if ws == 1:
                # the early copy: hashes + nBits as soon as hb_jobs and the side stream are done, at
                # the end of the side stream itself and issued after every full-hash launch. Streams
                # share the process's 4 hardware queues: a kernel queued behind this copy's event
                # waits sat out the side stream (the second epoch range's launch started 450 us
                # late), and a copy queued behind a full-hash launch waited for it (profiles/README
                # r5z)
                h.stream_wait_event(s0, self.ev_jobs)
                h.memcpy_async(self.early_host.data_ptr(), out + n, n * 36, s0, "dtoh")
                h.event_record(self.ev_early, s0)
            h.stream_wait_event(s, self.ev_side[0])
            if ws == 1:  # the early copy reads `out` and lands in early_host: both done before ev_end
                h.stream_wait_event(s, self.ev_early)
            if ws > 1:
                self._gather(world, n, per, lo_r, hi_r)
            h.memcpy_async(self.out_host.data_ptr(), out, n * 37, s, "dtoh")
            h.event_record(self.ev_end, s)
        t_issue = time.perf_counter()
        if overlap is not None:
            def early():
                if ws != 1:
                    return None
                h.event_synchronize(self.ev_early)
                e = self.early_host.numpy()
                return e[:n * 32].reshape(n, 32), e[n * 32:n * 36].view("<u4")

            overlap(early)
        t_overlap = time.perf_counter()
        h.event_synchronize(self.ev_end)
        t_done = time.perf_counter()
        res = self.out_host.numpy()
        return {"codes": res[:n], "hashes": res[n:n * 33].reshape(n, 32), "bits": res[n * 33:n * 37].view("<u4"),
                "pack_ms": (t_pack - t0) * 1e3, "issue_ms": (t_issue - t_pack) * 1e3,
                "overlap_ms": (t_overlap - t_issue) * 1e3, "wait_ms": (t_done - t_overlap) * 1e3,
                "device_ms": h.event_elapsed_ms(self.ev_start, self.ev_end)}

    def _gather(self, world, n: int, per: int, lo_r: int, hi_r: int) -> None:
        """All ranks' codes and block hashes (33 bytes per row) into every rank's result buffer:
        one all_gather_into_tensor of per x 33 bytes per rank, RCCL over xGMI device to device
        (the DGW nBits are computed by every rank for the whole batch: nothing to exchange)."""
        import torch.distributed as dist

        ws = world.world_size
        cnt = hi_r - lo_r
        send = self.gath[ws * per * 33: ws * per * 33 + per * 33].view(per, 33)
        if cnt:
            send[:cnt, 0] = self.out[lo_r:hi_r]
            send[:cnt, 1:] = self.out[n + lo_r * 32:n + hi_r * 32].view(cnt, 32)
        recv = self.gath[:ws * per * 33]
        dist.all_gather_into_tensor(recv, send.reshape(-1), group=world.group)
        g = recv.view(ws, per, 33)
        for r in range(ws):
            lo, hi = min(n, r * per), min(n, (r + 1) * per)
            if hi > lo:
                self.out[lo:hi] = g[r, :hi - lo, 0]
                self.out[n + lo * 32:n + hi * 32] = g[r, :hi - lo, 1:].reshape(-1)
