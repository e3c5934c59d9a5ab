#!/bin/bash
# r3d: GPU tier (new headline-epoch / pipelined-loop tests), smoke, the bench through the node's
# mining loop, and the bench's corrupted-DAG hook (must exit non-zero on the share re-hash).
set -o pipefail
mkdir -p gpurun_out/r3d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3d/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3d/bench.json 2> gpurun_out/r3d/bench.err &&
{ timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --equihash 0 --verify 0 --corrupt-dag \
    > gpurun_out/r3d/bench_corrupt.json 2> gpurun_out/r3d/bench_corrupt.err; echo "corrupt_rc=$?" >> gpurun_out/r3d/bench_corrupt.err; }
echo "exit=$?"
