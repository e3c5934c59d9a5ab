#!/usr/bin/env python3
"""Runs tools/jump_table_probe.hip (prebuilt to tools/jt.hsaco): the jump-table math / merge
dispatch on 256 lanes per kind, each launch synchronised, against a host reference. One JSON line."""
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rotl(x, r):
    r &= 31
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF if r else x


def math_ref(a, b, k):
    M = 0xFFFFFFFF
    clz = lambda x: 32 - x.bit_length()  # noqa: E731
    return [(a + b) & M, (a * b) & M, (a * b) >> 32, min(a, b), rotl(a, b), rotl(a, (32 - (b & 31)) & 31),
            a & b, a | b, a ^ b, clz(a) + clz(b), bin(a).count("1") + bin(b).count("1")][min(k, 10)]


def merge_ref(a, b, k, r):
    M = 0xFFFFFFFF
    return [(a * 33 + b) & M, ((a ^ b) * 33) & M, rotl(a, r) ^ b, rotl(a, (32 - (r & 31)) & 31) ^ b][k & 3]


def main() -> int:
    import numpy as np
    import torch

    from nodexa_chain_core_amd.ops import runtime

    co = runtime.load_code_object(os.path.join(os.path.dirname(os.path.abspath(__file__)), "jt.hsaco"))
    km, kg = co.function("jt_math"), co.function("jt_merge")
    rng = np.random.default_rng(3)
    a = rng.integers(0, 2**32, 256, dtype=np.uint64).astype(np.uint32)
    b = rng.integers(0, 2**32, 256, dtype=np.uint64).astype(np.uint32)
    a[:4] = [0, 1, 0xFFFFFFFF, 0x80000000]
    b[:4] = [0, 0xFFFFFFFF, 33, 1]
    da = torch.from_numpy(a.view(np.int32)).cuda()
    db = torch.from_numpy(b.view(np.int32)).cuda()
    out = torch.empty(256, dtype=torch.int32, device="cuda")
    s = runtime.current_stream_handle()
    bad = []
    for k in range(16):
        km.launch((1, 1, 1), (256, 1, 1), 0, s, struct.pack("<QQQI4x", da.data_ptr(), db.data_ptr(), out.data_ptr(), k))
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        if any(int(got[i]) != math_ref(int(a[i]), int(b[i]), k) for i in range(256)):
            bad.append(("math", k))
    for k in range(4):
        for r in (0, 1, 5, 31, 37):
            kg.launch((1, 1, 1), (256, 1, 1), 0, s,
                      struct.pack("<QQQII", da.data_ptr(), db.data_ptr(), out.data_ptr(), k, r))
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            if any(int(got[i]) != merge_ref(int(a[i]), int(b[i]), k, r) for i in range(256)):
                bad.append(("merge", k, r))
    print(json.dumps({"jump_table_ok": not bad, "bad": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
