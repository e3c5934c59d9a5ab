#!/bin/bash
# r3y: rehearsal of the restored tree: GPU tier, smoke, driver-contract bench (KawPow via the node's
# mining loop + Equihash + config-5 verify), then kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out/r3y
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3y/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3y/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3y/bench.json 2> gpurun_out/r3y/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r3y/prof -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/r3y/prof.log 2>&1
echo "exit=$?"
