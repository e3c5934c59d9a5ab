#!/bin/bash
# r3g: the pointer-path (DAG >= 4 GiB) variants after the LDS-occupancy fix, and where the bench's
# Equihash time goes.
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 400 python -u tools/kawpow_sweep.py --epoch 390 --rounds 5 --variants tuned tuned+KP_PRIO KP_HASHES=1,KP_DPP,KP_BARRETT,KP_L1X4,KP_NT_DAG,KP_SCHED_FENCE,KP_BLOCK=512,KP_MIN_WAVES=4,KP_DIGEST_REG KP_HASHES=1,KP_DPP,KP_BARRETT,KP_L1X4,KP_NT_DAG,KP_SCHED_FENCE,KP_BLOCK=512,KP_MIN_WAVES=4,KP_DIGEST_REG,KP_PRIO \
  --out gpurun_out/r3g/sweep390.json > gpurun_out/r3g/sweep390.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --verify 0 > gpurun_out/r3g/bench.json 2> gpurun_out/r3g/bench.err &&
timeout -k 10 300 python -u tools/equihash_bench.py > gpurun_out/r3g/equihash_bench.log 2>&1
echo "exit=$?"
