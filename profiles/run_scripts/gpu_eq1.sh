#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_equihash.py -x -q > gpurun_out/pytest_eq.log 2>&1
echo "pytest exit=$?" >> gpurun_out/pytest_eq.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --equihash 8 > gpurun_out/bench2.log 2>&1
echo "bench exit=$?"
