#!/bin/bash
# r3a: random 256 B gather ceiling (KawPow DAG pattern) + GPU tier sanity on the round-3 start tree.
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 120 tools/bin/gather_ceiling > gpurun_out/r3a/gather_ceiling.jsonl 2> gpurun_out/r3a/gather_ceiling.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r3a/pytest_gpu.log 2>&1
echo "exit=$?"
