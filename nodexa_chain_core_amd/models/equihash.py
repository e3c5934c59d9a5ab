"""Equihash(200,9) front-end: header extension, solving and verification.

The reference has no Equihash: this is the engine's new,
opt-in extension (Appendix D). Consensus input for a header is

    I = CKAWPOWInput-style 80 bytes (version, prev, merkle, time, bits, height)
        || nonce256 (32 bytes)                         -> 112 bytes

and the solution (512 x 21-bit indices, 1344 bytes) travels after the header as
CompactSize || bytes, only on networks whose `equihash_activation_time` has
passed (UINT32_MAX — never — on main/test/regtest as shipped).
"""
from __future__ import annotations

import os
import struct
import time

from .. import _core

PARAMS = _core.EquihashParams(200, 9)


def header_input(header, nonce256: bytes) -> bytes:
    """I for a chain.header.BlockHeader / _core.BlockHeader and a 32-byte nonce."""
    if len(nonce256) != 32:
        raise ValueError("nonce256 must be 32 bytes")
    base = struct.pack("<i32s32sIII", header.version, header.prev, header.merkle_root, header.time, header.bits,
                       header.height)
    return base + nonce256


def solve_cpu(inp: bytes, max_solutions: int = 16) -> list[list[int]]:
    sols, _ = _core.equihash_solve_cpu(PARAMS, inp, max_solutions, 0)
    return sols


def verify(inp: bytes, solution: bytes | list[int]) -> bool:
    idx = _core.equihash_unpack(PARAMS, solution) if isinstance(solution, (bytes, bytearray)) else list(solution)
    return bool(_core.equihash_verify(PARAMS, inp, idx)[0])


def pack(indices: list[int]) -> bytes:
    return _core.equihash_pack(PARAMS, indices)


def bench_device(num_batches: int = 4, num_inst: int = 8, warmup: int = 1) -> float:
    """Sol/s of the GPU solver on random 112-byte inputs (all solutions host-verified)."""
    import torch

    from ..ops.equihash import EquihashSolver

    solver = EquihashSolver(num_inst=num_inst)
    rng = os.urandom
    batches = [[rng(112) for _ in range(num_inst)] for _ in range(num_batches + warmup)]
    for b in batches[:warmup]:
        solver.solve(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    total = 0
    for b in batches[warmup:]:
        solver.launch(b)
        total += sum(len(s) for s in solver.collect(b))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return total / dt
