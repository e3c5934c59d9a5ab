#!/bin/bash
# r2c: private-slot Equihash engine (equihash_ps.hip) vs the global-slot engine.
set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 300 python -u -m pytest tests/test_gpu_equihash.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r2c/pytest_eq.log 2>&1 &&
timeout -k 10 300 python -u tools/equihash_bench.py --inst 8 --batches 6 --engines global ps ps:64 ps:256 \
  > gpurun_out/r2c/bench.jsonl 2>&1
echo "exit=$?"
