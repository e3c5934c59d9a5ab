#!/bin/bash
# r2w: GPU tier, smoke and bench on the last commit of the round.
set -o pipefail
mkdir -p gpurun_out/r2w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2w/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2w/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r2w/bench.json 2> gpurun_out/r2w/bench.err
echo "exit=$?"
