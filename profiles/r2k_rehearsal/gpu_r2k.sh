#!/bin/bash
# r2k: rehearsal after the container rebuild (fresh in-tree build): GPU tier, smoke, bench.
set -o pipefail
mkdir -p gpurun_out/r2k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2k/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2k/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r2k/bench.json 2> gpurun_out/r2k/bench.err
echo "exit=$?"
