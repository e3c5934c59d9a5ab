#!/bin/bash
# r3j: Equihash PS rows packed to the level's payload (7,7,6,5,5,4,4,3,2 words): exactness,
# fallback counters, device time per batch and per-kernel time.
set -o pipefail
mkdir -p gpurun_out/r3j
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_equihash.py -v --timeout 300 > gpurun_out/r3j/pytest_eq.log 2>&1 &&
timeout -k 10 300 python -u tools/eq_fallback_probe.py 24 > gpurun_out/r3j/eq_probe.log 2>&1 &&
timeout -k 10 300 python -u tools/equihash_bench.py --engines ps --batches 8 > gpurun_out/r3j/equihash_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3j/prof -o eq -- python3 tools/equihash_bench.py --engines ps --batches 4 > gpurun_out/r3j/prof.log 2>&1
echo "exit=$?"
