#!/bin/bash
# r2e: whole GPU tier + smoke + driver bench with the private-slot Equihash engine as default,
# plus the engine A/B and a kernel-trace profile of both engines.
set -o pipefail
mkdir -p gpurun_out/r2e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2e/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2e/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r2e/bench.log 2>&1 &&
timeout -k 10 300 python -u tools/equihash_bench.py --inst 8 --batches 8 --engines global ps \
  > gpurun_out/r2e/eq_engines.jsonl 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2e/prof -o eq -- python3 tools/equihash_bench.py --inst 8 --batches 3 --engines ps global > gpurun_out/r2e/prof.log 2>&1
echo "exit=$?"
