#!/bin/bash
# r3u: rehearsal of the restored tree: GPU tier, smoke, driver-contract bench (KawPow via the node's
# mining loop + Equihash + config-5 verify), then kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out/r3u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3u/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3u/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3u/bench.json 2> gpurun_out/r3u/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r3u/prof -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/r3u/prof.log 2>&1
echo "exit=$?"
