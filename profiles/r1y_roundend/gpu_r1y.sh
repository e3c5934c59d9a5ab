#!/bin/bash
# Round-end rehearsal: the whole GPU test tier, smoke(), and the 1-GPU driver bench.
set -o pipefail
mkdir -p gpurun_out/${OUT:-r1y}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${OUT:-r1y}/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${OUT:-r1y}/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/${OUT:-r1y}/bench.log 2>&1
echo "exit=$?"
