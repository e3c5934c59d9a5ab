#!/bin/bash
# r2h: block connection through the GPU signature batch + the whole GPU test tier.
set -o pipefail
mkdir -p gpurun_out/r2h
timeout -k 10 300 python -u -m pytest tests/test_gpu_block_sigs.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2h/pytest_block_sigs.log 2>&1 &&
timeout -k 10 300 python -u tools/block_connect_bench.py --txs 8000 --threads 16 --reps 3 --gpu \
  > gpurun_out/r2h/block_connect.jsonl 2> gpurun_out/r2h/block_connect.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2h/pytest_gpu_all.log 2>&1
echo "exit=$?"
