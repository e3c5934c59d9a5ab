"""Equihash(200,9) solver on one MI355X.

`EquihashSolver(num_inst)` solves `num_inst` inputs (different nonces) per launch sequence — 1
BLAKE2b generation kernel, 8 collision rounds, the final 40-bit round and the index
reconstruction, all enqueued on one stream with no host synchronisation in between — and checks
every solution on the device (equihash.hip eq_verify_slots) before it is reported.

The engine is the private-slot solver (equihash_ps.hip): every workgroup owns a segment of
every destination bucket, so a row costs one LDS atomic and one store. Two alternatives were
built, measured and removed: one global atomic per row (equihash.hip until round 5: 6.5 ms per
8 solves against 4.4) and coarse destination buckets with the fine bucket bits in the row
(equihash_cb.hip in round 5: fewer EA write requests per row, 0.38-0.77 against 1.0-1.27, but
9.3-12.7 ms per 16-solve window against 8.5 — the producers' extra staging work cost more than
the stores saved; profiles/README r5a-r5e). Memory per instance: 2 x 4096 x 2048 x 32 B row
buffers (537 MB of address space, ~67 MB written per level) + 9 levels of index refs (151 MB).
"""
from __future__ import annotations

import struct

import numpy as np
import torch

from .. import _core
from ..utils.trace import traced
from . import runtime

KERNELS = ["eqp_gen"] + [f"eqp_round{r}" for r in range(1, 9)] + ["eqp_final", "eqp_reconstruct"]


def blake2b_h0(n: int = 200, k: int = 9) -> list[int]:
    """BLAKE2b initial chaining value for digest (512/n)*n/8 bytes and the Zcash personal."""
    iv = [0x6a09e667f3bcc908, 0xbb67ae8584caa73b, 0x3c6ef372fe94f82b, 0xa54ff53a5f1d36f1,
          0x510e527fade682d1, 0x9b05688c2b3e6c1f, 0x1f83d9abfb41bd6b, 0x5be0cd19137e2179]
    param = bytearray(64)
    param[0] = (512 // n) * n // 8
    param[2] = 1
    param[3] = 1
    param[48:56] = b"ZcashPoW"
    param[56:60] = struct.pack("<I", n)
    param[60:64] = struct.pack("<I", k)
    words = struct.unpack("<8Q", bytes(param))
    return [a ^ b for a, b in zip(iv, words)]


def pack_solutions(sols: np.ndarray) -> list[bytes]:
    """(m, 512) leaf indices -> m packed 1344-byte solutions (512 x 21-bit big-endian), vectorised
    (the same bytes as _core.equihash_pack)."""
    sols = np.ascontiguousarray(np.asarray(sols, dtype=np.uint32).reshape(-1, 512))
    be = (sols << np.uint32(11)).astype(">u4").view(np.uint8).reshape(-1, 512, 4)
    bits = np.unpackbits(be, axis=2)[:, :, :21].reshape(len(sols), 512 * 21)
    packed = np.packbits(bits, axis=1)
    return [r.tobytes() for r in packed]


@traced("equihash.verify")
def verify_solutions(inputs: list[bytes], solutions: list[bytes], device: int | None = None) -> list[bool]:
    """GPU batch check of packed (n=200, k=9) solutions (hip/kernels/equihash.hip eq_verify):
    one workgroup per solution. `inputs` are the 112-byte header inputs."""
    if len(inputs) != len(solutions):
        raise ValueError("inputs and solutions differ in length")
    runtime.require_gpu()
    h = runtime.hip()
    n = len(inputs)
    out_ok = [False] * n
    good = [i for i in range(n) if len(solutions[i]) == 4 * h.EQ_SOL_WORDS and len(inputs[i]) <= 124]
    if not good:
        return out_ok
    lens = {len(inputs[i]) for i in good}
    if len(lens) != 1:
        raise ValueError("one input length per batch")
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else int(device))
    msgs = bytearray(len(good) * 128)
    sols = bytearray(len(good) * 4 * h.EQ_SOL_WORDS)
    for k, i in enumerate(good):
        msgs[k * 128:k * 128 + len(inputs[i])] = inputs[i]
        sols[k * 4 * h.EQ_SOL_WORDS:(k + 1) * 4 * h.EQ_SOL_WORDS] = solutions[i]
    with torch.cuda.device(dev):
        kern = runtime.static_kernel("equihash", "eq_verify")
        dm = torch.frombuffer(msgs, dtype=torch.int64).to(dev)
        ds = torch.frombuffer(sols, dtype=torch.int32).to(dev)
        res = torch.full((len(good),), -1, dtype=torch.int32, device=dev)
        h.launch_equihash_verify(kern, blake2b_h0(), dm.data_ptr(), lens.pop(), len(good), ds.data_ptr(),
                                 res.data_ptr(), runtime.current_stream_handle())
        verdicts = res.cpu().tolist()
    for k, i in enumerate(good):
        out_ok[i] = verdicts[k] == 0
    return out_ok


class EquihashSolver:
    def __init__(self, num_inst: int = 8, device: int | None = None, code_object: str | None = None,
                 groups: int | None = None, block: int = 1024, final_groups: int | None = None):
        """`code_object`: path of an alternative build of equihash_ps.hip (tuning sweeps);
        `groups` writers (workgroups) per instance per round, by default so that groups x
        instances = 256 (one 1024-thread workgroup per CU)."""
        runtime.require_gpu()
        self.h = runtime.hip()
        # writers per instance: one 1024-thread workgroup per CU over the whole launch (P x
        # instances = 256: 32 at 8 instances, 16 at the mining window's 16; profiles/README r4k:
        # 8.50 vs 8.65 ms at 16 instances, and 7.48 vs 4.38 ms when P=16 leaves half the CUs idle at 8)
        self.groups = int(groups) if groups else min(256, max(16, 1 << max(0, (256 // max(1, int(num_inst))).bit_length() - 1)))
        self.block = int(block)  # threads per workgroup, must match the code object's EQP_BLOCK
        # final round (writes no level, so any width works): ~4096 workgroups over the launch
        # (256 at 16 instances: -1 % against 1024, r4k)
        self.final_groups = int(final_groups or 0) or min(1024, max(64, 4096 // max(1, int(num_inst))))
        self.num_inst = int(num_inst)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else int(device))
        self.params = _core.EquihashParams(200, 9)
        B, L = self.h.EQ_BUCKETS, self.h.EQ_LEVELS
        ni = self.num_inst
        with torch.cuda.device(self.device):
            if code_object is None:
                self.kernels = [runtime.static_kernel("equihash_ps", k) for k in KERNELS]
            else:
                co = runtime.load_code_object(code_object)
                self.kernels = [co.function(k) for k in KERNELS]
            S, R, W = self.h.EQP_SLOTS, self.h.EQP_REF_STRIDE, self.h.EQ_WORDS
            self.hashes = torch.empty(2 * ni * B * S * W, dtype=torch.int32, device=self.device)
            self.refs = torch.empty(ni * L * B * R, dtype=torch.int32, device=self.device)
            self.counts = torch.empty(ni * L * self.groups * B, dtype=torch.uint8, device=self.device)
            self.stats_buf = torch.zeros(ni * self.h.EQP_STATS, dtype=torch.int32, device=self.device)
            self.cands = torch.empty(ni * (1 + 2 * self.h.EQ_MAX_CAND), dtype=torch.int32, device=self.device)
            self.sols = torch.empty(ni * (1 + self.h.EQ_MAX_SOL * 512), dtype=torch.int32, device=self.device)
            self.msgs = torch.zeros(ni * 16, dtype=torch.int64, device=self.device)
            # two pinned landing buffers: the solutions of launch i are copied
            # back on the stream right after its kernels, so launch i+1 can be
            # queued before the host verifies launch i (GPU and CPU overlap)
            self._landing = [torch.empty(self.sols.numel(), dtype=torch.int32).pin_memory() for _ in range(2)]
            # per launch: [inst][EQP_STATS] truncation counters + [inst] candidate counts
            nstat = ni * self.h.EQP_STATS
            self._land_stats = [torch.zeros(nstat + ni, dtype=torch.int32).pin_memory() for _ in range(2)]
            # device-side check of every solution slot (equihash.hip eq_verify_slots) right after the
            # solve: the verdicts ride back with the solutions, so collect() needs no host pass over
            # the 512 leaves of each solution (~225 us per solution on one core)
            self.verify_kernel = runtime.static_kernel("equihash", "eq_verify_slots")
            self.verdicts = torch.empty(ni * self.h.EQ_MAX_SOL, dtype=torch.int32, device=self.device)
            self._land_verdicts = [torch.empty(ni * self.h.EQ_MAX_SOL, dtype=torch.int32).pin_memory()
                                   for _ in range(2)]
            self.fallbacks = 0  # instances re-solved on the host because the device truncated something
            self.fallback_log: list[dict] = []
            self._stage = [torch.empty(ni * 16, dtype=torch.int64).pin_memory() for _ in range(2)]
        self._pending: list[tuple[list[bytes], torch.Tensor, torch.cuda.Event]] = []
        self._next = 0
        self.h0 = blake2b_h0()
        self.input_len = None

    def launch(self, inputs: list[bytes], stream: int | None = None) -> None:
        if len(inputs) != self.num_inst:
            raise ValueError(f"need exactly {self.num_inst} inputs")
        lens = {len(x) for x in inputs}
        if len(lens) != 1 or next(iter(lens)) > 124 or next(iter(lens)) % 4:
            raise ValueError("inputs must share one length <= 124 bytes, multiple of 4")
        self.input_len = next(iter(lens))
        if len(self._pending) >= len(self._landing):
            raise RuntimeError("collect() the oldest launch before queueing another")
        buf = bytearray(self.num_inst * 128)
        for i, x in enumerate(inputs):
            buf[i * 128:i * 128 + len(x)] = x
        with torch.cuda.device(self.device):
            # staged through pinned memory so the upload is stream-ordered and the
            # host does not wait for the previous launch (slot reuse is safe: its
            # previous copy completed before that launch's landing event)
            stage = self._stage[self._next]
            stage.copy_(torch.frombuffer(buf, dtype=torch.int64))
            self.msgs.copy_(stage, non_blocking=True)
            s = runtime.current_stream_handle() if stream is None else stream
            self.h.launch_equihash_ps_solve(self.kernels, self.h0, self.msgs.data_ptr(), self.input_len, self.num_inst,
                                            self.groups, self.hashes.data_ptr(), self.refs.data_ptr(),
                                            self.counts.data_ptr(), self.cands.data_ptr(), self.sols.data_ptr(),
                                            self.stats_buf.data_ptr(), s, self.block, self.final_groups)
            self.h.launch_equihash_verify_slots(self.verify_kernel, self.h0, self.msgs.data_ptr(), self.input_len,
                                                self.num_inst, self.sols.data_ptr(), self.verdicts.data_ptr(), s)
            land = self._landing[self._next]
            lstat = self._land_stats[self._next]
            lver = self._land_verdicts[self._next]
            self._next = (self._next + 1) % len(self._landing)
            land.copy_(self.sols, non_blocking=True)
            lver.copy_(self.verdicts, non_blocking=True)
            nstat = lstat.numel() - self.num_inst
            lstat[:nstat].copy_(self.stats_buf, non_blocking=True)
            lstat[nstat:].copy_(self.cands.view(self.num_inst, -1)[:, 0], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self._pending.append((list(inputs), (land, lstat, lver), ev))

    def _lossy(self, st: np.ndarray) -> bool:
        """Whether one instance's stats row records a loss: segment / staging overflow or a cut
        chain (slots 0-10); slot 11 is a diagnostic maximum."""
        return bool(st[:self.h.EQP_STAT_STAGE + 1].any())

    def collect_arrays(self, inputs: list[bytes] | None = None, verify: str = "device") -> list[np.ndarray]:
        """Solutions of the oldest queued launch (waits only for that launch), one (m, 512) uint32
        array of leaf indices per instance. verify: "device" (the eq_verify_slots verdicts that came
        back with the launch), "host" (the C++ golden verifier as well) or "none". A solution that
        fails is a solver bug and raises."""
        if not self._pending:
            raise RuntimeError("nothing launched")
        launched, (land, lstat, lver), ev = self._pending.pop(0)
        if inputs is not None and list(inputs) != launched:
            raise ValueError("collect() inputs differ from the oldest launch")
        inputs = launched
        ev.synchronize()
        ms = self.h.EQ_MAX_SOL
        raw = land.numpy()
        per = 1 + ms * 512
        st = lstat.numpy()
        verdicts = lver.numpy().reshape(self.num_inst, ms)
        nstat = st.size - self.num_inst
        out = []
        for i in range(self.num_inst):
            truncated = int(st[nstat + i]) > self.h.EQ_MAX_CAND
            truncated |= self._lossy(st[i * self.h.EQP_STATS:(i + 1) * self.h.EQP_STATS])
            if truncated:
                # a bucket, chain or candidate cap cut something: the device result may miss a
                # solution, so this instance is solved again on the golden solver (it keeps the
                # solution set exact by construction)
                self.fallbacks += 1
                self.fallback_log.append({"stats": st[i * self.h.EQP_STATS:(i + 1) * self.h.EQP_STATS].tolist(),
                                          "candidates": int(st[nstat + i])})
                sols, _ = _core.equihash_solve_cpu(self.params, inputs[i], ms, 0)
                out.append(np.asarray(sols, dtype=np.uint32).reshape(-1, 512))
                continue
            base = i * per
            n = min(int(raw[base]), ms)
            sols = raw[base + 1: base + 1 + n * 512].view(np.uint32).reshape(n, 512)
            if verify != "none" and n:
                bad = np.flatnonzero(verdicts[i, :n] != 0)
                if len(bad):
                    raise RuntimeError(f"GPU produced an invalid Equihash solution for instance {i} "
                                       f"(device verdict {int(verdicts[i, bad[0]])})")
            if verify == "host":
                for s in range(n):
                    if not _core.equihash_verify(self.params, inputs[i], sols[s].tolist())[0]:
                        raise RuntimeError(f"GPU produced an invalid Equihash solution for instance {i}")
            if n > 1:  # distinct solutions only (the reconstruct stage may emit one tree twice)
                _, first = np.unique(sols, axis=0, return_index=True)
                sols = sols[np.sort(first)]
            out.append(np.array(sols))
        return out

    def collect(self, inputs: list[bytes] | None = None, verify: bool = True) -> list[list[list[int]]]:
        """collect_arrays() as lists of index lists; verify=True also runs the host verifier."""
        return [a.tolist() for a in self.collect_arrays(inputs, "host" if verify else "device")]

    @traced("equihash.solve")
    def solve(self, inputs: list[bytes]) -> list[list[list[int]]]:
        self.launch(inputs)
        return self.collect(inputs)

    def stats(self) -> dict:
        """Per-level fill of the last solve (instance 0) — overflow diagnostics."""
        B, L = self.h.EQ_BUCKETS, self.h.EQ_LEVELS
        c = self.counts[: L * self.groups * B].view(L, self.groups, B).to(torch.int32).sum(1).cpu()
        dropped = self.stats_buf[: self.h.EQP_STATS].cpu().tolist()
        return {"rows_per_level": [int(x) for x in c.sum(1)], "max_fill": [int(x) for x in c.max(1).values],
                "cap": self.h.EQP_STAGE, "dropped_per_level": dropped[:L],
                "stage_dropped": dropped[self.h.EQP_STAT_STAGE], "largest_bucket": dropped[self.h.EQP_STAT_STAGE_MAX],
                "chains_cut": dropped[self.h.EQP_STAT_CHAIN], "candidates": int(self.cands[0].item())}
