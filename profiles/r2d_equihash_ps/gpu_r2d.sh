#!/bin/bash
# r2d: private-slot Equihash engine (pipelined rounds, 16-byte rows from level 5) vs the global engine.
set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 300 python -u -m pytest tests/test_gpu_equihash.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r2d/pytest_eq.log 2>&1 &&
timeout -k 10 300 python -u tools/equihash_bench.py --inst 8 --batches 6 --engines global ps:64 ps:128 ps:32 \
  > gpurun_out/r2d/bench.jsonl 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2d/prof -o eq -- python3 tools/equihash_bench.py --inst 8 --batches 3 --engines ps global > gpurun_out/r2d/prof.log 2>&1
echo "exit=$?"
