#!/bin/bash
# Round-1 re-entry check: GPU tests, smoke, headline bench, batch-verify bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1d
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1d/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1d/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r1d/bench.log 2>&1 && \
timeout -k 10 400 python tools/verify_bench.py --cpu-sample 20 > gpurun_out/r1d/verify_bench.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
