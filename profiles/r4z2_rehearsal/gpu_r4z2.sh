#!/bin/bash
# r4z2: second round-end rehearsal of the round-4 tree: the whole GPU tier, smoke(), the driver-contract
# bench (KawPow through the node loop + Equihash through the node loop + config-5 verify), then a
# kernel trace of a short bench.
set -o pipefail
mkdir -p gpurun_out/r4z2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r4z2/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4z2/smoke.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r4z2/bench.json 2> gpurun_out/r4z2/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r4z2/prof -o bench --output-format csv \
  -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/r4z2/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4z2/prof_verify -o v --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --equihash 0 --verify 1 > gpurun_out/r4z2/prof_verify.log 2>&1
echo "exit=$?"
