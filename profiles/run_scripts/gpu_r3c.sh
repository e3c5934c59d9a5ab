#!/bin/bash
# r3c: KawPow search variants — scheduling fences around the round program, rolled keccak-f800
set -o pipefail
mkdir -p gpurun_out/r3c
V='tuned+KP_SCHED_FENCE tuned-KP_DIGEST_REG+KP_DIGEST_GLOBAL+KP_SCHED_FENCE tuned+KP_SCHED_FENCE+KP_SCHED_ILP tuned+KP_SCHED_FENCE-KP_BLOCK=768-KP_MIN_WAVES=6+KP_BLOCK=512+KP_MIN_WAVES=4 tuned+KP_SCHED_FENCE-KP_NT_DAG tuned'
timeout -k 10 500 python -u tools/kawpow_sweep.py --rounds 7 --variants $V --out gpurun_out/r3c/sweep384.json > gpurun_out/r3c/sweep384.log 2>&1
echo "exit=$?"
