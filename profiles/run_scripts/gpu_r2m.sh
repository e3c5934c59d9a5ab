#!/bin/bash
# r2m: occupancy ladder with register-resident digests: 640 / 768 / 896-thread workgroups
# (5 / 6 / 7 waves per SIMD, two workgroups per CU on the 64 KiB L1 table), epoch 384.
set -o pipefail
mkdir -p gpurun_out/r2m
timeout -k 10 600 python -u tools/kawpow_sweep.py --epoch 384 --rounds 7 --out gpurun_out/r2m/sweep384.jsonl \
  --variants tuned \
  "tuned-KP_BLOCK=512+KP_BLOCK=640+KP_DIGEST_REG+KP_MIN_WAVES=5" \
  "tuned-KP_BLOCK=512+KP_BLOCK=768+KP_DIGEST_REG+KP_MIN_WAVES=6" \
  "tuned-KP_BLOCK=512+KP_BLOCK=896+KP_DIGEST_REG+KP_MIN_WAVES=7" \
  > gpurun_out/r2m/sweep384.log 2>&1
echo "exit=$?"
