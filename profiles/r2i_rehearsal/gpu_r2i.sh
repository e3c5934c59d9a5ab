#!/bin/bash
# r2i: round-end style rehearsal after the UTXO / asset / index work: GPU tier, smoke, bench.
set -o pipefail
mkdir -p gpurun_out/r2i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2i/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2i/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r2i/bench.json 2> gpurun_out/r2i/bench.err
echo "exit=$?"
