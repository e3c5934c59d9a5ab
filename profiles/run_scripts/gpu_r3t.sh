#!/bin/bash
# r3t: Equihash PS new default (1024 threads, 448 producers, 32 writers): exactness, fallbacks,
# per-kernel time; two 1024-thread workgroups per CU (64-VGPR build) vs one.
set -o pipefail
mkdir -p gpurun_out/r3t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_equihash.py -v --timeout 200 > gpurun_out/r3t/pytest_eq.log 2>&1 &&
timeout -k 10 200 python -u tools/eq_fallback_probe.py 24 > gpurun_out/r3t/eq_probe.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps ps:64 --batches 6 --variants "" EQP_MIN_WAVES=8 EQP_NP=384,EQP_MIN_WAVES=8 > gpurun_out/r3t/eb.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps:64:512 ps:128:512 --batches 6 --variants EQP_BLOCK=512,EQP_NP=256,EQP_MIN_WAVES=8 >> gpurun_out/r3t/eb.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t/prof -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 4 > gpurun_out/r3t/prof.log 2>&1
echo "exit=$?"
