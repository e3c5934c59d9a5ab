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


@pytest.mark.parametrize("n,launcher", [(1, "none"), (2, "torchrun"), (8, "torchrun"), (2, "self"), (8, "self")])
def test_bench_contract_on_cpu(n, launcher):
    """n = 8: the driver's whole-node launch shape (8 ranks, one JSON line with n_gpus 8), both under
    torchrun and as a bare `bench.py --gpus 8` (bench.py starts its own ranks)."""
    args = ["bench.py", "--gpus", str(n), "--device", "cpu", "--epoch", "0", "--steps", "2", "--warmup", "1",
            "--batch", "4", "--equihash", "0", "--verify", "0", "--quiet"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == f"dp{n}" and out["config"]["global_batch"] == 4 * n
    assert out["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert out["shares_rehashed"] > 0 and "MiningService" in out["loop"]


def test_bench_refuses_world_size_mismatch():
    """A launcher that started a different number of ranks than --gpus asks for: exit 2, no line."""
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--device", "cpu", "--quiet"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "WORLD_SIZE=4" in r.stderr and not r.stdout.strip()


def test_bench_self_launch_propagates_rank_failure():
    """A rank that fails makes the whole self-launched run fail (the other ranks are ended)."""
    args = ["bench.py", "--gpus", "2", "--device", "cpu", "--epoch", "0", "--steps", "2", "--warmup", "1",
            "--batch", "4", "--equihash", "0", "--verify", "0", "--quiet"]
    env = dict(os.environ, OMP_NUM_THREADS="1", NODEXA_BENCH_FAIL_RANK="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_bench_self_launch_sigterm_takes_ranks_down():
    """The launcher stopped with SIGTERM (a driver timeout) ends its rank processes too."""
    import signal
    import time

    import psutil

    args = ["bench.py", "--gpus", "2", "--device", "cpu", "--epoch", "0", "--steps", "100000", "--warmup", "1",
            "--batch", "4", "--equihash", "0", "--verify", "0", "--quiet"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.Popen([sys.executable] + args, cwd=ROOT, env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL)
    try:
        deadline = time.time() + 120
        kids = []
        while time.time() < deadline and len(kids) < 2:
            kids = psutil.Process(p.pid).children()
            time.sleep(0.2)
        assert len(kids) == 2
        time.sleep(2)
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) != 0
        gone, alive = psutil.wait_procs(kids, timeout=60)
        assert not alive
    finally:
        if p.poll() is None:
            p.kill()
