#!/bin/bash
# Full GPU check of the current tree: all GPU tests, smoke, headline bench, kernel stats of the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1l
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r1l/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1l/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r1l/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1l/prof -o bench -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/r1l/prof_bench.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
