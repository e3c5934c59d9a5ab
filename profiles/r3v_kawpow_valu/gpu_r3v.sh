#!/bin/bash
# r3v: KawPow variants after the fence: branch-free 24-bit Barrett for the item index (two
# quarter-rate multiplies off the gather's critical path), the shift form of a*33, both.
set -o pipefail
mkdir -p gpurun_out/r3v
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 500 python -u tools/kawpow_sweep.py --rounds 7 --variants tuned tuned+KP_FASTMOD24 tuned+KP_MUL33_SHIFT tuned+KP_FASTMOD24+KP_MUL33_SHIFT tuned+KP_FASTMOD24+KP_PRIO \
  --out gpurun_out/r3v/sweep384.json > gpurun_out/r3v/sweep384.log 2>&1
echo "exit=$?"
