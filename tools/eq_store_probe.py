#!/usr/bin/env python3
"""Launch the Equihash private-slot solver N times without collecting (a build whose results may be
invalid, e.g. EQP_NO_ROW_STORE, must not reach the verifiers): for counter runs under rocprofv3.

    python tools/eq_store_probe.py [--variant EQP_NO_ROW_STORE] [--inst 16] [--launches 2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="")
    ap.add_argument("--inst", type=int, default=16)
    ap.add_argument("--launches", type=int, default=2)
    a = ap.parse_args()
    import torch

    from equihash_bench import variant_object
    from nodexa_chain_core_amd.ops.equihash import EquihashSolver

    defines = tuple(x for x in a.variant.split(",") if x)
    s = EquihashSolver(num_inst=a.inst, code_object=variant_object(defines, "equihash_ps.hip"))
    s.hashes.zero_()
    for k in range(a.launches):
        s.launch([bytes([k, j]) * 56 for j in range(a.inst)])
        torch.cuda.synchronize()
        s._pending.clear()  # results deliberately not collected
    print("launched", a.launches, "x", a.inst, "instances", defines or "(base)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
