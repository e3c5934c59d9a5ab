#!/bin/bash
# r3r: Equihash PS with 1024-thread workgroups and 32 writers per level (half the segment-line
# footprint at the same waves per CU).
set -o pipefail
mkdir -p gpurun_out/r3r
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python -u tools/equihash_bench.py --engines ps --batches 6 --variants "" > gpurun_out/r3r/eb.log 2>&1 &&
timeout -k 10 300 python -u tools/equihash_bench.py --engines ps:32:1024 --batches 6 --variants EQP_BLOCK=1024 EQP_BLOCK=1024,EQP_NP=128 EQP_BLOCK=1024,EQP_NP=384 >> gpurun_out/r3r/eb.log 2>&1 &&
timeout -k 10 300 python -u tools/equihash_bench.py --engines ps:64:1024 --batches 6 --variants EQP_BLOCK=1024 >> gpurun_out/r3r/eb.log 2>&1
echo "exit=$?"
