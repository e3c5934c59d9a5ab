#!/bin/bash
# Round-end rehearsal: the whole GPU test suite, smoke(), and the 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out/r1q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r1q/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1q/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r1q/bench.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
