#!/bin/bash
# r3s: Equihash PS producer/consumer split and workgroup size sweep.
set -o pipefail
mkdir -p gpurun_out/r3s
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps --batches 6 --variants "" EQP_NP=192 EQP_NP=256 > gpurun_out/r3s/eb.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps:32:1024 --batches 6 --variants EQP_BLOCK=1024,EQP_NP=384 EQP_BLOCK=1024,EQP_NP=448 EQP_BLOCK=1024,EQP_NP=512 >> gpurun_out/r3s/eb.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps:32:768 ps:64:768 --batches 6 --variants EQP_BLOCK=768,EQP_NP=256 EQP_BLOCK=768,EQP_NP=320 >> gpurun_out/r3s/eb.log 2>&1
echo "exit=$?"
