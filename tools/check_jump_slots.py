#!/usr/bin/env python3
"""CLI of nodexa_chain_core_amd/ops/jump_slots.py (the kawpow_verify_waves handler-slot check).

    python tools/check_jump_slots.py nodexa_chain_core_amd/kernels/kawpow_verify_light.hsaco
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nodexa_chain_core_amd.ops.jump_slots import LLVM, check  # noqa: E402,F401

if __name__ == "__main__":
    r = check(sys.argv[1])
    print(json.dumps(r))
    sys.exit(1 if r["n_errors"] or not (r["tables"] or r["inline_sites"]) else 0)
