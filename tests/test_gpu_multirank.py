"""The N>1 bench path on the GPU: two torchrun ranks share GPU 0 and exchange over gloo (RCCL
refuses two ranks on one device), so the driver's multi-GPU run — DAG built half per rank and
all-gathered, the mining loop's work-packet broadcast and share all-gather, the resident header
verify sliced over the ranks and all-gathered, MAX-over-ranks timing, one JSON line from rank 0 — is
exercised on every GPU tier, not only on an 8-GPU node
(profiles/README r3za)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("launcher", ["torchrun", "self"])
def test_two_rank_bench_on_one_gpu(gpu, launcher):
    """launcher "self": a bare `bench.py --gpus 2` starts its own two ranks (the driver's N-GPU run
    need not wrap the bench in torchrun)."""
    # torchrun: the resident verify split over the ranks (shard threshold 0); self: the default
    # policy, where the 10k batch is verified by rank 0 and the verdict broadcast
    env = dict(os.environ, NODEXA_DIST_BACKEND="gloo", NODEXA_VERIFY_SHARD_MIN="0" if launcher == "torchrun" else "65536")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    pre = [sys.executable]
    if launcher == "torchrun":
        pre += ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port())]
    cmd = pre + ["bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", str(1 << 23),
                 "--equihash", "2", "--verify", "1", "--check-shares", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] % 2 == 0 and out["value"] > 0
    assert out["shares_rehashed"] >= 1  # re-hashed in full on the host, 0 mismatches (else exit 1)
    assert out["equihash_sol_per_s"] > 0
    # the resident verify sliced over the ranks, codes + block hashes all-gathered (header_batch._gather)
    assert out["verify_headers_per_s"] > 0 and out["verify_headers_light_per_s"] > 0
    assert out["verify_headers"]["resident"]["ranks"].startswith("split" if launcher == "torchrun" else "rank 0")
    assert "over 2 GPU(s)" in r.stderr  # the DAG was built sharded and all-gathered
