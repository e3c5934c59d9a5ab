"""gfx950 X16R / X16RV2 batch hashing (hip/kernels/x16r.hip) vs the reference-derived chain
vectors and the host implementation."""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VEC = json.load(open(os.path.join(os.path.dirname(__file__), "data", "x16r_vectors.json")))


def test_reference_chain_vectors(core, gpu):
    from nodexa_chain_core_amd.ops.x16r import x16r_hash_batch

    hdrs = b"".join(bytes.fromhex(c["header"]) for c in VEC["chains"])
    for v2, key in ((False, "x16r"), (True, "x16rv2")):
        got = x16r_hash_batch(hdrs, v2=v2)
        assert [bytes(r).hex() for r in got] == [c[key] for c in VEC["chains"]]


def test_random_batch_mixed_versions_vs_host(core, gpu):
    from nodexa_chain_core_amd.ops.x16r import x16r_hash_batch

    rng = random.Random(3)
    n = 1500
    hdrs = [rng.randbytes(80) for _ in range(n)]
    v2 = np.array([rng.random() < 0.5 for _ in range(n)])
    got = x16r_hash_batch(b"".join(hdrs), v2=v2)
    for i in range(0, n, 7):  # the host chain is the slow side
        fn = core.x16rv2 if v2[i] else core.x16r
        assert bytes(got[i]) == fn(hdrs[i], hdrs[i][4:36]), i
