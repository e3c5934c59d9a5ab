#!/bin/bash
# r3w: 8 waves/SIMD — 1024-thread workgroups at 64 VGPRs (digests parked in HBM or held in
# registers), against the 768-thread / 6-wave default.
set -o pipefail
mkdir -p gpurun_out/r3w
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 500 python -u tools/kawpow_sweep.py --rounds 7 --variants tuned \
  tuned-KP_BLOCK=768-KP_DIGEST_REG-KP_MIN_WAVES=6+KP_BLOCK=1024+KP_DIGEST_GLOBAL+KP_MIN_WAVES=8 \
  tuned-KP_BLOCK=768-KP_MIN_WAVES=6+KP_BLOCK=1024+KP_MIN_WAVES=8 \
  tuned-KP_DIGEST_REG+KP_DIGEST_GLOBAL \
  --out gpurun_out/r3w/sweep384.json > gpurun_out/r3w/sweep384.log 2>&1
echo "exit=$?"
