"""The X16R / X16RV2 device primitives (hip/kernels/x16r_device.hpp), compiled for the host.

The gfx950 kernel (hip/kernels/x16r.hip) runs these functions per lane; here the same header is
built with g++ (X16R_FN = inline) into a throwaway shared object and checked against the host
implementation (csrc/pow/x16r*.cpp, itself pinned to the reference's sph sources by
tests/test_x16r.py) for every slot at the two input lengths the chain uses (the 80-byte header,
then 64-byte digests), and against the reference-derived chain vectors of tests/data/x16r_vectors.json.
The GPU tier runs the kernel itself (tests/test_gpu_x16r.py)."""
import ctypes
import json
import os
import random
import shutil
import subprocess

import pytest

from nodexa_chain_core_amd import core

_core = core()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "nodexa_chain_core_amd", "hip", "kernels")
VEC = json.load(open(os.path.join(os.path.dirname(__file__), "data", "x16r_vectors.json")))

_HARNESS = r"""
#include <stdint.h>
#define X16R_FN inline
#include "x16r_device.hpp"
extern "C" void dev_single(int algo, const uint8_t* in, int n, uint8_t* out) { x16rd::single(algo, in, n, out); }
extern "C" void dev_chain(const uint8_t* header80, int v2, uint8_t* out32) {
    uint8_t a[80], b[64];
    for (int i = 0; i < 80; ++i) a[i] = header80[i];
    int len = 80;
    for (int s = 0; s < 16; ++s) {
        x16rd::step(x16rd::selection(header80 + 4, s), v2 != 0, a, len, b);
        for (int i = 0; i < 64; ++i) a[i] = b[i];
        len = 64;
    }
    for (int i = 0; i < 32; ++i) out32[i] = a[i];
}
"""


@pytest.fixture(scope="module")
def dev(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    d = tmp_path_factory.mktemp("x16r_dev")
    src, so = d / "h.cpp", d / "h.so"
    src.write_text(_HARNESS)
    subprocess.run([cxx, "-O1", "-std=c++17", "-shared", "-fPIC", "-I", KDIR, str(src), "-o", str(so)], check=True)
    lib = ctypes.CDLL(str(so))
    return lib


def _single(lib, algo, data):
    out = ctypes.create_string_buffer(64)
    lib.dev_single(algo, data, len(data), out)
    return out.raw


@pytest.mark.parametrize("slot", range(17))
def test_device_primitive_matches_host(dev, slot):
    rng = random.Random(100 + slot)
    for n in (64, 80):
        for _ in range(4):
            d = rng.randbytes(n)
            assert _single(dev, slot, d) == _core.x16r_algo(slot, d), (slot, n)


def test_device_chain_matches_reference_vectors(dev):
    for c in VEC["chains"]:
        hdr = bytes.fromhex(c["header"])
        for v2, key in ((0, "x16r"), (1, "x16rv2")):
            out = ctypes.create_string_buffer(32)
            dev.dev_chain(hdr, v2, out)
            assert out.raw.hex() == c[key]


def test_generated_tables_are_current(tmp_path):
    """x16r_tables.inc is what tools/x16r_gen_tables.cpp emits from the host sources today."""
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "gen"
    csrc = os.path.join(ROOT, "nodexa_chain_core_amd", "csrc")
    subprocess.run([cxx, "-O1", "-std=c++17", "-I", csrc, os.path.join(ROOT, "tools", "x16r_gen_tables.cpp"),
                    os.path.join(csrc, "crypto", "keccak.cpp"), os.path.join(csrc, "util", "common.cpp"),
                    "-o", str(exe)], check=True)
    got = subprocess.run([str(exe)], check=True, capture_output=True).stdout
    assert got == open(os.path.join(KDIR, "x16r_tables.inc"), "rb").read()
