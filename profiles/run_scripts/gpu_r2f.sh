#!/bin/bash
# r2f: Equihash private-slot engine with the final round over 1024 workgroups per instance.
set -o pipefail
mkdir -p gpurun_out/r2f
timeout -k 10 300 python -u -m pytest tests/test_gpu_equihash.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r2f/pytest_eq.log 2>&1 &&
timeout -k 10 300 python -u tools/equihash_bench.py --inst 8 --batches 8 --engines global ps \
  > gpurun_out/r2f/eq_engines.jsonl 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2f/prof -o eq -- python3 tools/equihash_bench.py --inst 8 --batches 3 --engines ps > gpurun_out/r2f/prof.log 2>&1
echo "exit=$?"
