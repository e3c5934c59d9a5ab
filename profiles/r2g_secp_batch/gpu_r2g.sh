#!/bin/bash
# r2g: GPU batch ECDSA verification — correctness vs the golden model and throughput.
set -o pipefail
mkdir -p gpurun_out/r2g
timeout -k 10 300 python -u -m pytest tests/test_secp_batch.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r2g/pytest_secp.log 2>&1 &&
timeout -k 10 300 python -u tools/secp_bench.py > gpurun_out/r2g/secp_bench.jsonl 2>&1
echo "exit=$?"
