"""The in-tree build (nodexa_chain_core_amd/_build.py) as a fresh GPU box and a torchrun job see it.

A gpurun snapshot (and the driver's box) carries the built .so files but not build/: with every
output newer than its sources the build must do nothing, not recompile and relink under the
processes that load the libraries. The ranks of a torchrun job all call it at once: one builds,
the others wait on the lock."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fresh_outputs_need_no_objects(tmp_path, monkeypatch):
    from nodexa_chain_core_amd import _build

    _build.build_core()  # up to date (conftest built it)
    so = os.path.join(_build.PKG, "_core" + _build.EXT)
    before = os.stat(so).st_mtime_ns
    monkeypatch.setattr(_build, "BUILD", str(tmp_path / "obj"))  # as on a box without build/
    _build.build_core()
    assert os.stat(so).st_mtime_ns == before
    assert not (tmp_path / "obj").exists()


def test_lock_is_reentrant():
    from nodexa_chain_core_amd import _build

    with _build._build_lock():
        with _build._build_lock():
            assert _build._LOCK_DEPTH == 2
    assert _build._LOCK_DEPTH == 0


def test_concurrent_builds():
    code = ("from nodexa_chain_core_amd import _build; _build.build_core(); "
            "from nodexa_chain_core_amd import _core; print(_core.sha256d(b'x').hex())")
    procs = [subprocess.Popen([sys.executable, "-c", code], cwd=ROOT, stdout=subprocess.PIPE, text=True)
             for _ in range(4)]
    outs = [p.communicate(timeout=600)[0].strip() for p in procs]
    assert all(p.returncode == 0 for p in procs)
    assert len(set(outs)) == 1 and len(outs[0]) == 64
