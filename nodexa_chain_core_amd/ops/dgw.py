"""Batch DarkGravityWave on the GPU (hip/kernels/dgw.hip).

`expected_bits` turns the (nTime, nBits) series of a linear header batch
(`HeaderChain.dgw_series`: up to 180 ancestors then the batch) into the nBits every header must
carry, one GPU thread per header. The result goes to `HeaderChain.accept_headers(bits=...)`, so
the host's contextual stage keeps only the serial index updates. Bit-exact with the host's
dgw_average (csrc/chain/pow_rules.cpp), the reference's DarkGravityWave (src/pow.cpp:18-102);
tests/test_gpu_verify.py compares the two over the 10k-header fixture."""
from __future__ import annotations

import numpy as np
import torch

from .. import core
from . import runtime

_core = core()


def expected_bits(params, times: bytes, bits: bytes, a: int, n: int, base_height: int, device: int = 0) -> np.ndarray:
    """(n,) uint32 expected nBits; 0 where the header is not a DGW header (the host decides)."""
    if n == 0:
        return np.zeros(0, np.uint32)
    if len(times) != 4 * (a + n) or len(bits) != 4 * (a + n):
        raise ValueError("series must hold a + n u32 values")
    c = _core.dgw_constants(params)
    dev = torch.device("cuda", device)
    with torch.cuda.device(device):
        d_t = torch.from_numpy(np.frombuffer(times, dtype=np.int32).copy()).to(dev)
        d_b = torch.from_numpy(np.frombuffer(bits, dtype=np.int32).copy()).to(dev)
        d_o = torch.empty(n, dtype=torch.int32, device=dev)
        runtime.hip().launch_dgw(runtime.static_kernel("dgw", "dgw_batch"), d_t.data_ptr(), d_b.data_ptr(),
                                 d_o.data_ptr(), a, n, base_height, c["dgw_activation_block"], c["kawpow_time"],
                                 c["equihash_time"], c["limits"], c["compacts"], c["target_timespan"],
                                 runtime.current_stream_handle())
        return d_o.cpu().numpy().view(np.uint32)


def batch_bits(chain, headers, hashes_blob: bytes, device: int = 0) -> bytes | None:
    """The `bits` argument of accept_headers for a batch, computed on the GPU, or None when the
    batch has no DGW series (not linear, or a network without DGW retargeting)."""
    s = chain.dgw_series(headers, hashes_blob)
    if s is None:
        return None
    times, bits, a, base = s
    return expected_bits(chain.params, times, bits, a, len(headers), base, device).tobytes()
