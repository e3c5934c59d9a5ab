"""Synthetic header chains with real proof of work and real retargeting.

BASELINE config 5 verifies "10k synthetic KawPow+Equihash headers + DarkGravityWave";
there is no chain data in this environment, so this module mines one:
  * testnet rules (DGW from block 1, 180-block window, pow limit 2^248 — ~256
    hashes per header) with the KawPow activation moved to genesis+1, so every
    header is a 120-byte KawPow header;
  * optionally an Equihash(200,9) era after `n_kawpow` headers (the new header
    extension, csrc/chain/primitives.hpp): extended headers with a 32-byte nonce
    and a 1344-byte solution, DGW bootstrapping the era from the Equihash limit;
  * note: DGW multiplies a 256-bit average target by the timespan without overflow
    protection (src/pow.cpp:93-94, reproduced bit-exactly), so with testnet's 2^248
    limit the first post-bootstrap retarget wraps and the difficulty jumps; an
    Equihash era is therefore kept inside its 180-block bootstrap window;
  * block times jittered around the 60 s target so DGW actually retargets; the mean
    spacing is 61 s because DGW measures 179 intervals against a 180-interval
    timespan, so an exact 60 s mean would ratchet the difficulty up block after block.
Each header's proof of work is found by search:
  * backend "cpu": the golden models (`_core.kawpow_search_full` over a lazily
    filled host DAG; `_core.equihash_solve_cpu`) — small chains for tests;
  * backend "gpu": the DAG-resident batch kernel (ops/verify.py) as a
    period-agnostic KawPow searcher, and the gfx950 Equihash solver.
The chain is accepted header by header into a C++ HeaderChain (contextual
checks + DGW) while it is built, so every header in the output is valid.
Files: concatenated serialized headers + `<file>.json` with the parameters.
"""
from __future__ import annotations

import json
import os
import random

from .. import core
from ..chain.header import from_progpow, to_progpow
from ..chain.state import make_params

_core = core()


def synthetic_params(network: str = "test", equihash_activation_time: int | None = None):
    g = _core.make_chain_params(network)
    return make_params(network, kawpow_activation_time=int(g.genesis.header.time) + 1,
                       equihash_activation_time=equihash_activation_time)


def _boundary(bits: int) -> bytes:
    target, neg, ovf = _core.set_compact(bits)
    return target.to_bytes(32, "big") if not (neg or ovf) else bytes(32)


def _target(bits: int) -> int:
    target, neg, ovf = _core.set_compact(bits)
    return 0 if (neg or ovf) else target


class _CpuKawpow:
    def __init__(self, threads: int = 0):
        self.threads = threads or (os.cpu_count() or 4)
        self.dags: dict[int, object] = {}

    def __call__(self, height: int, header_hash: bytes, boundary: bytes, start: int):
        epoch = height // _core.EPOCH_LENGTH
        dag = self.dags.get(epoch)
        if dag is None:
            dag = self.dags[epoch] = _core.HostDag(_core.get_epoch_context(epoch))
        ok, nonce, fin, mix = _core.kawpow_search_full(dag, height, header_hash, boundary, start, 512, self.threads)
        return ((nonce, fin, mix) if ok else None), 512


class _GpuKawpow:
    # One scanner launch costs ~5.6 ms at 2048 nonces and is latency-bound (each
    # 16-lane group hashes its 16 jobs serially), so a 32k window costs about the
    # same and covers the post-bootstrap DGW difficulty in one call.
    def __init__(self, device: int = 0, width: int = 32768):
        from ..ops.verify import DagNonceScanner

        self.scan = DagNonceScanner(device, width)

    def __call__(self, height: int, header_hash: bytes, boundary: bytes, start: int):
        return self.scan(height, header_hash, boundary, start)


class _CpuEquihash:
    batch = 1

    def solve(self, inputs: list[bytes]) -> list[list[list[int]]]:
        p = _core.EquihashParams(200, 9)
        return [_core.equihash_solve_cpu(p, x, 16, 0)[0] for x in inputs]  # (solutions, stats)


class _GpuEquihash:
    batch = 8

    def __init__(self, device: int = 0):
        from ..ops.equihash import EquihashSolver

        self.solver = EquihashSolver(num_inst=8, device=device)

    def solve(self, inputs: list[bytes]) -> list[list[list[int]]]:
        return self.solver.solve(inputs)


def _solve_equihash_header(h, params, solver, rng) -> None:
    """Search nonce256 values until a solution's SHA256d(header) meets nBits."""
    p = _core.EquihashParams(params.equihash_n, params.equihash_k)
    target = _target(h.bits)
    act = params.kawpow_activation_time
    while True:
        nonces = [rng.getrandbits(256).to_bytes(32, "little") for _ in range(solver.batch)]
        inputs = []
        for nn in nonces:
            h.nonce256 = nn
            inputs.append(h.equihash_input())
        for nn, sols in zip(nonces, solver.solve(inputs)):
            for sol in sols:
                h.nonce256 = nn
                h.solution = _core.equihash_pack(p, sol)
                if int.from_bytes(h.equihash_hash(act), "little") <= target:
                    return


ANCHOR_LEN = 181  # stored headers below a fixture that starts past genesis: DGW reads 180, MTP 11


def make_anchor(params, first_height: int, end_time: int, seed: int = 1):
    """The stored headers a node has below height `first_height` (HeaderChain.add_anchor): ANCHOR_LEN
    linked KawPow-layout headers at the pow limit, 61 s apart, the last at `end_time`, plus the
    chain work below them (genesis, then the pow-limit proof per block). Their proof of work is not checked (a
    loaded block index is not re-validated), so they are not mined. Returns (headers, base_height,
    base_work)."""
    base = first_height - ANCHOR_LEN
    if base <= 0:
        raise ValueError("an anchored fixture starts above height ANCHOR_LEN")
    limit_bits = _core.HeaderChain(params).next_bits(params.genesis.header)  # height 1: the pow limit
    chain = _core.HeaderChain(params)
    out, prev = [], bytes(32)
    for k in range(ANCHOR_LEN):
        h = _core.BlockHeader()
        h.version = 0x30000000
        h.prev = prev
        h.merkle_root = _core.sha256d(b"nodexa-anchor-%d-%d" % (seed, base + k))
        h.time = end_time - 61 * (ANCHOR_LEN - 1 - k)
        h.height = base + k
        h.bits = limit_bits
        h.nonce64 = k
        out.append(h)
        prev = chain.block_hash(h)
    target, _, _ = _core.set_compact(limit_bits)
    work = (1 << 256) // (target + 1)
    # genesis' work (testnet genesis is harder than the pow limit) + the pow-limit proof per block
    return out, base, int(chain.genesis().chain_work) + work * (base - 1)


def build_chain(n_kawpow: int, n_equihash: int = 0, network: str = "test", backend: str = "cpu", seed: int = 1,
                device: int = 0, spacing: tuple[int, int] = (21, 101), progress=None, first_height: int = 1):
    """Mine `n_kawpow` KawPow headers then `n_equihash` Equihash-extension headers on top of
    `network`'s genesis, or (first_height > 1) on top of a make_anchor run ending at
    first_height - 1 (a node's stored index at that height: the headline-epoch fixture starts at
    2,880,000, epoch 384). Returns (params, headers); with an anchor, (params, headers, anchor)."""
    rng = random.Random(seed)
    base = synthetic_params(network)
    t0 = int(base.genesis.header.time) + 61 * (first_height - 1)
    times, t = [], t0
    for _ in range(n_kawpow + n_equihash):
        t += rng.randint(*spacing)
        times.append(t)
    eq_act = times[n_kawpow] if n_equihash else None
    params = synthetic_params(network, eq_act)
    chain = _core.HeaderChain(params)
    anchor = None
    if first_height > 1:
        anchor = make_anchor(params, first_height, t0, seed)
        chain.add_anchor(*anchor)
    kp = _GpuKawpow(device) if backend == "gpu" else _CpuKawpow()
    eq = (_GpuEquihash(device) if backend == "gpu" else _CpuEquihash()) if n_equihash else None
    out = []
    for i in range(1, n_kawpow + n_equihash + 1):
        height = first_height - 1 + i
        h = _core.BlockHeader()
        h.version = 0x30000000 | (_core.EQUIHASH_VERSION_BIT if i > n_kawpow else 0)
        h.prev = chain.tip().hash
        h.merkle_root = _core.sha256d(b"nodexa-synthetic-%d-%d" % (seed, height))
        h.time = times[i - 1]
        h.height = height
        h.bits = chain.next_bits(h)
        if i <= n_kawpow:
            hh = to_progpow(h.kawpow_header_hash())
            boundary = _boundary(h.bits)
            start = rng.getrandbits(40) << 16
            found = None
            while found is None:
                found, tried = kp(height, hh, boundary, start)
                start += tried
            nonce, fin, mix = found
            h.nonce64 = nonce
            h.mix_hash = from_progpow(mix)
        else:
            _solve_equihash_header(h, params, eq, rng)
        r = chain.accept_header(h, h.time + 7200, i > n_kawpow)  # Equihash era: full check while mining
        if not r.ok:
            raise RuntimeError(f"synthetic header {height} rejected: {r.reject}")
        out.append(h)
        if progress and (i % 250 == 0 or (i > n_kawpow and i % 10 == 0)):  # Equihash headers are ~100x slower
            progress(i)
    return (params, out) if anchor is None else (params, out, anchor)


def build_kawpow_chain(n: int, network: str = "test", backend: str = "cpu", seed: int = 1, device: int = 0,
                       spacing: tuple[int, int] = (21, 101), progress=None):
    return build_chain(n, 0, network, backend, seed, device, spacing, progress)


def save(path: str, params, headers, anchor=None) -> None:
    """`path`: the headers, serialized back to back; `path`.json: parameters; with an anchor
    (make_anchor), `path`.anchor holds its headers and the json its height and chain work."""
    act = params.kawpow_activation_time
    with open(path, "wb") as f:
        for h in headers:
            f.write(h.serialize(act))
    meta = {"network": params.network_id, "kawpow_activation_time": int(params.kawpow_activation_time),
            "equihash_activation_time": int(params.equihash_activation_time), "headers": len(headers),
            "equihash_headers": sum(1 for h in headers if h.is_equihash())}
    if anchor is not None:
        ahs, base_height, base_work = anchor
        with open(path + ".anchor", "wb") as f:
            for h in ahs:
                f.write(h.serialize(act))
        meta.update({"first_height": int(headers[0].height), "anchor_height": base_height,
                     "anchor_headers": len(ahs), "anchor_work": hex(base_work)})
    with open(path + ".json", "w") as f:
        json.dump(meta, f, indent=1)


def load(path: str):
    with open(path + ".json") as f:
        meta = json.load(f)
    eq = meta["equihash_activation_time"]
    params = make_params(meta["network"], kawpow_activation_time=meta["kawpow_activation_time"],
                         equihash_activation_time=None if eq == 0xFFFFFFFF else eq)
    with open(path, "rb") as f:
        headers = _core.deserialize_headers(f.read(), params.kawpow_activation_time)
    if len(headers) != meta["headers"]:
        raise ValueError("header count mismatch")
    return params, headers


def load_anchor(path: str, params):
    """The fixture's anchor (make_anchor) as (headers, base_height, base_work), or None."""
    with open(path + ".json") as f:
        meta = json.load(f)
    if "anchor_height" not in meta:
        return None
    with open(path + ".anchor", "rb") as f:
        hs = _core.deserialize_headers(f.read(), params.kawpow_activation_time)
    if len(hs) != meta["anchor_headers"]:
        raise ValueError("anchor header count mismatch")
    return hs, int(meta["anchor_height"]), int(meta["anchor_work"], 16)


def new_chain(params, anchor=None):
    """A HeaderChain for verifying a fixture: genesis, plus the fixture's anchor when it has one."""
    chain = _core.HeaderChain(params)
    if anchor is not None:
        chain.add_anchor(*anchor)
    return chain
