#!/bin/bash
# r3k: Equihash PS with aligned row padding; does a larger batch (more resident workgroups) pay?
set -o pipefail
mkdir -p gpurun_out/r3k
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_equihash.py -v --timeout 200 -k "ps" > gpurun_out/r3k/pytest_eq.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps --batches 8 --inst 8 > gpurun_out/r3k/eb8.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps --batches 6 --inst 16 > gpurun_out/r3k/eb16.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps --batches 4 --inst 32 > gpurun_out/r3k/eb32.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps:128 --batches 6 --inst 16 > gpurun_out/r3k/eb16_128.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k/prof -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 4 > gpurun_out/r3k/prof.log 2>&1
echo "exit=$?"
