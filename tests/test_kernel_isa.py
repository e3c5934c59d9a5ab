"""Checks on the built gfx950 code (CPU only: disassembly of the in-tree code objects).

kawpow_verify_waves dispatches its ProgPoW ops through a table of 64-byte handler slots
(hip/kernels/kawpow_verify_light.hip, kwt_table): a slot that does not start with its kind's handler
would send a wave into the middle of another instruction, so the layout the assembler produced is
checked slot by slot (ops/jump_slots.py) before any GPU run loads it."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HSACO = os.path.join(ROOT, "nodexa_chain_core_amd", "kernels", "kawpow_verify_light.hsaco")
SRC = os.path.join(ROOT, "nodexa_chain_core_amd", "hip", "kernels", "kawpow_verify_light.hip")




def _tools():
    return os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump") and os.path.exists(
        "/opt/rocm/lib/llvm/bin/clang-offload-bundler")


@pytest.mark.skipif(not _tools(), reason="ROCm LLVM tools not installed")
def test_verify_waves_handler_slots(tmp_path):
    from nodexa_chain_core_amd.ops.jump_slots import check

    path = HSACO
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(SRC):
        if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
            pytest.skip("kernel not built and no hipcc")
        path = str(tmp_path / "kvl.hsaco")
        subprocess.run(["/opt/rocm/bin/hipcc", "--genco", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-mcode-object-version=5", "-I", os.path.dirname(SRC), SRC, "-o", path], check=True)
    r = check(path)
    assert r["n_errors"] == 0, r["errors"]
    assert r["tables"] == 1  # one table, in kawpow_verify_waves
    assert r["calls"] == 33  # per round: 11 cache merges, 18 math ops, 4 DAG merges


def test_slot_stamp_fails_closed(tmp_path):
    """The loader only takes a kawpow_verify_light code object whose stamp matches its bytes: a
    changed code object (or one built where the check could not run) is refused before any load."""
    from nodexa_chain_core_amd.ops import jump_slots, runtime

    if not os.path.exists(HSACO):
        pytest.skip("kernel not built")
    assert jump_slots.stamp_ok(HSACO)  # _build.build_kernels stamped the shipped one
    kdir = tmp_path / "kernels"
    kdir.mkdir()
    bad = kdir / "kawpow_verify_light.hsaco"
    raw = bytearray(open(HSACO, "rb").read())
    raw[-1] ^= 1
    bad.write_bytes(bytes(raw))
    open(jump_slots.stamp_path(str(bad)), "w").write(open(jump_slots.stamp_path(HSACO)).read())
    assert not jump_slots.stamp_ok(str(bad))
    old = runtime.KERNEL_DIR
    runtime.KERNEL_DIR = str(kdir)
    try:
        with pytest.raises(runtime.NativeUnavailable, match="stamp"):
            runtime.static_kernel("kawpow_verify_light", "kawpow_verify_waves")
    finally:
        runtime.KERNEL_DIR = old
