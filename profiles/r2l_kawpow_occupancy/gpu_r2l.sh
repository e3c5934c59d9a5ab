#!/bin/bash
# r2l: register-resident digests (KP_DIGEST_REG) and the occupancy they unlock (768 / 1024-thread
# workgroups with only the 64 KiB L1 table in LDS), epoch 384, interleaved A/B.
set -o pipefail
mkdir -p gpurun_out/r2l
timeout -k 10 600 python -u tools/kawpow_sweep.py --epoch 384 --rounds 5 --out gpurun_out/r2l/sweep384.jsonl \
  --variants tuned tuned+KP_DIGEST_REG \
  "tuned-KP_BLOCK=512+KP_BLOCK=768+KP_DIGEST_REG+KP_MIN_WAVES=6" \
  "tuned-KP_BLOCK=512+KP_BLOCK=1024+KP_DIGEST_REG+KP_MIN_WAVES=8" \
  > gpurun_out/r2l/sweep384.log 2>&1
echo "exit=$?"
