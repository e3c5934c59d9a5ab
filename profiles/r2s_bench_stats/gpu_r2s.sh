#!/bin/bash
# r2s: rocprofv3 kernel statistics of the driver-contract bench (768-thread KawPow default, 2^25
# nonces per step, Equihash private-slot engine).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2s
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s -o bench -- \
  python3 bench.py --steps 10 --warmup 2 > gpurun_out/r2s/bench.json 2> gpurun_out/r2s/bench.err
echo "exit=$?"
