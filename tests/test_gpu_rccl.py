"""RCCL for real on a 1-GPU box: a one-rank "nccl" process group (parallel/world.init
force_collectives) runs every collective of the sharded DAG build, the mining loop (with an injected
collective failure -> ncclCommAbort -> new communicator) and batch verify as RCCL kernels
(tests/rccl_one_rank.py, in a fresh process)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_one_rank_rccl_world(gpu, tmp_path):
    out = tmp_path / "rccl.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29000 + os.getpid() % 1000),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", TORCH_NCCL_ASYNC_ERROR_HANDLING="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_one_rank.py"), str(out)], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-5000:])
    rep = json.load(open(out))
    assert rep["backend"] == "nccl" and rep["world_size"] == 1 and rep["collective"]
    assert rep["hashes_before_abort"] > 0 and rep["hashes_total"] > rep["hashes_before_abort"]
    assert rep["injected"] and "injected" in rep["injected"]  # the failure path ran
    assert rep["steps_after_abort"] >= rep["steps_before_abort"] + 6  # mined on after the abort
    assert rep["shares_checked"] >= 1 and rep["share_mismatches"] == 0
    assert rep["verify_equal"] and rep["verify_valid"] == 2000
