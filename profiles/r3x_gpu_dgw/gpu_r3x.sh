#!/bin/bash
# r3x: GPU DarkGravityWave batch kernel (bit-exactness vs the host rules over both 10k fixtures)
# and the batch-verify stage times of the bench with it.
set -o pipefail
mkdir -p gpurun_out/r3x
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py -v --timeout 200 --timeout-method thread \
  > gpurun_out/r3x/pytest_gpu_verify.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --equihash 2 > gpurun_out/r3x/bench.json 2> gpurun_out/r3x/bench.err
echo "exit=$?"
