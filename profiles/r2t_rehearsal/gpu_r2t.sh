#!/bin/bash
# r2t: final rehearsal of the round: GPU tier, smoke, bench (driver contract defaults).
set -o pipefail
mkdir -p gpurun_out/r2t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2t/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2t/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r2t/bench.json 2> gpurun_out/r2t/bench.err
echo "exit=$?"
