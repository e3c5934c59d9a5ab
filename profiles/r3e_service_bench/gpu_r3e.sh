#!/bin/bash
# r3e: GPU tier + smoke + bench (node's mining loop) + corrupted-DAG bench hook, then KawPow sweeps:
# wave priority on the DAG critical path, max-ILP scheduler, and the fence at epoch 390 (pointer path).
set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3e/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3e/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3e/bench.json 2> gpurun_out/r3e/bench.err &&
{ timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --equihash 0 --verify 0 --corrupt-dag \
    > gpurun_out/r3e/bench_corrupt.json 2> gpurun_out/r3e/bench_corrupt.err; echo "corrupt_rc=$?" >> gpurun_out/r3e/bench_corrupt.err; } &&
timeout -k 10 400 python -u tools/kawpow_sweep.py --rounds 7 --variants tuned tuned+KP_PRIO tuned+KP_SCHED_ILP tuned+KP_PRIO+KP_SCHED_ILP tuned-KP_SCHED_FENCE \
  --out gpurun_out/r3e/sweep384.json > gpurun_out/r3e/sweep384.log 2>&1 &&
timeout -k 10 400 python -u tools/kawpow_sweep.py --epoch 390 --rounds 5 --variants tuned tuned-KP_SCHED_FENCE tuned+KP_PRIO \
  --out gpurun_out/r3e/sweep390.json > gpurun_out/r3e/sweep390.log 2>&1
echo "exit=$?"
