"""Device engines: ethash DAG, KawPow search/hash, Equihash, batch verify.

Importing this package imports torch first so that the HIP runtime torch
ships is the single one in the process (see ops/runtime.py).
"""
from . import runtime  # noqa: F401
