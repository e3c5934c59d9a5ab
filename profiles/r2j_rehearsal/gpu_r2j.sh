#!/bin/bash
# r2j: rehearsal after the wallet, messaging and rewards work: GPU tier, smoke, bench.
set -o pipefail
mkdir -p gpurun_out/r2j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2j/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2j/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r2j/bench.json 2> gpurun_out/r2j/bench.err
echo "exit=$?"
