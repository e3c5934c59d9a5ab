#!/bin/bash
# r2n: the 768-thread / register-digest default on the large-DAG pointer path (epoch 390) against
# the previous 512-thread default, then the GPU tier, smoke and bench with the new default.
set -o pipefail
mkdir -p gpurun_out/r2n
timeout -k 10 600 python -u tools/kawpow_sweep.py --epoch 390 --rounds 5 --out gpurun_out/r2n/sweep390.jsonl \
  --variants tuned "tuned-KP_BLOCK=768-KP_DIGEST_REG-KP_MIN_WAVES=6+KP_BLOCK=512" \
  > gpurun_out/r2n/sweep390.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2n/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2n/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r2n/bench.json 2> gpurun_out/r2n/bench.err
echo "exit=$?"
