"""nodexa_chain_core_amd — MI355X-native PoW mining and block-validation engine.

A from-scratch rebuild (not a port) of the capabilities of
DeonDavisV/Nodexa-Chain-Core (Clore/Ravencoin-derived node): KawPow
(ProgPoW 0.9.4 + RAVENCOINKAWPOW) and Ethash, X16R/X16RV2, DarkGravityWave,
the 80/120-byte header and blk?????.dat formats, the mining JSON-RPC surface,
plus a new Equihash(200,9) engine behind an opt-in header extension.

Layout
  csrc/      native C++ core (crypto, PoW golden models, consensus)   -> _core
  hip/       gfx950 kernels + HIP host runtime                         -> _hip, kernels/*.hsaco
  models/    PoW algorithm front-ends (kawpow, ethash, equihash, x16r)
  ops/       device-side engines (DAG, search, verify, JIT)
  parallel/  multi-GPU over RCCL (torch.distributed "nccl" backend)
  chain/     headers, blocks, params, DGW, block files
  rpc/       JSON-RPC server/client (reference-compatible method names)
  miner/     block templates, nonce scheduling, GPU miner controller
  utils/     config (ArgsManager syntax), logging, metrics
"""
__version__ = "0.1.0"


def core():
    """The native CPU core module (built in-tree by _build.py)."""
    from . import _core  # type: ignore[attr-defined]

    return _core
