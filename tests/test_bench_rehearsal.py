"""bench.py's driver contract rehearsed on CPU: the same mining loop and collectives as the GPU
run (miner/service.MiningService over gloo, CPU search devices), launched the way the driver
launches the N-GPU run (torch.distributed.run, one process per rank, 127.0.0.1 rendezvous)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n", [1, 2, 8])
def test_bench_contract_on_cpu(n):
    """n = 8: the driver's whole-node launch shape (8 ranks, one JSON line with n_gpus 8)."""
    args = ["bench.py", "--gpus", str(n), "--device", "cpu", "--epoch", "0", "--steps", "2", "--warmup", "1",
            "--batch", "4", "--equihash", "0", "--verify", "0", "--quiet"]
    if n > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == f"dp{n}" and out["config"]["global_batch"] == 4 * n
    assert out["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert out["shares_rehashed"] > 0 and "MiningService" in out["loop"]
