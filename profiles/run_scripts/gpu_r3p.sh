#!/bin/bash
# r3p: global-slot Equihash engine with XCD-local instances (bucket tails fill in one L2).
set -o pipefail
mkdir -p gpurun_out/r3p
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python -u tools/equihash_bench.py --engines global ps --banks 1 8 --batches 6 --variants "" EQ_XCD_MAP > gpurun_out/r3p/eb.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3p/prof -o eq --output-format csv -- python3 tools/equihash_bench.py --engines global --banks 1 --batches 4 --variants EQ_XCD_MAP > gpurun_out/r3p/prof.log 2>&1
echo "exit=$?"
