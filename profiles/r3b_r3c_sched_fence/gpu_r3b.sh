#!/bin/bash
# r3b: KawPow search variants — scheduling fences around the round program, rolled keccak-f800
# (register pressure), digests parked in HBM, 512 vs 768 threads. Interleaved, bit-exact checked.
set -o pipefail
mkdir -p gpurun_out/r3b
V='tuned tuned+KP_SCHED_FENCE+NX_KECCAK800_ROLLED tuned-KP_DIGEST_REG+KP_DIGEST_GLOBAL+KP_SCHED_FENCE+NX_KECCAK800_ROLLED tuned+KP_SCHED_FENCE tuned+NX_KECCAK800_ROLLED tuned-KP_BLOCK=768-KP_MIN_WAVES=6+KP_BLOCK=512+KP_MIN_WAVES=4+KP_SCHED_FENCE+NX_KECCAK800_ROLLED'
timeout -k 10 500 python -u tools/kawpow_sweep.py --rounds 7 --variants $V --out gpurun_out/r3b/sweep384.json > gpurun_out/r3b/sweep384.log 2>&1
echo "exit=$?"
