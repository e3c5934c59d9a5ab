#!/bin/bash
# r3t: Equihash PS two 1024-thread workgroups per CU (64-VGPR build) vs one.
set -o pipefail
mkdir -p gpurun_out/r3t
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps:32:1024 ps:64:1024 --batches 6 --variants EQP_BLOCK=1024,EQP_NP=448 EQP_BLOCK=1024,EQP_NP=448,EQP_MIN_WAVES=8 EQP_BLOCK=1024,EQP_NP=384,EQP_MIN_WAVES=8 > gpurun_out/r3t/eb.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps:64:512 ps:128:512 --batches 6 --variants EQP_BLOCK=512,EQP_NP=256,EQP_MIN_WAVES=8 >> gpurun_out/r3t/eb.log 2>&1
echo "exit=$?"
