#!/bin/bash
# r2r: GPU tier incl. the remote-mode miner, smoke, bench at the 2^25-nonce step.
set -o pipefail
mkdir -p gpurun_out/r2r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2r/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2r/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r2r/bench.json 2> gpurun_out/r2r/bench.err
echo "exit=$?"
