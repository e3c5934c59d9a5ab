#!/bin/bash
# Re-sweep of occupancy / cache-policy knobs around the current tuned KawPow variant (epoch 384).
set -o pipefail
mkdir -p gpurun_out/r1z
B="KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4"
# the r1z A/B: the pre-NT tuned variant (spelled out, since "tuned" now includes KP_NT_DAG) vs +NT
timeout -k 10 420 python -u tools/kawpow_sweep.py --epoch 384 --rounds 5 --variants "KP_HASHES=1,$B,KP_BLOCK=512" \
  "KP_HASHES=1,$B,KP_BLOCK=512,KP_NT_DAG" "KP_HASHES=1,$B,KP_BLOCK=256" "KP_HASHES=1,$B,KP_BLOCK=1024" \
  "KP_HASHES=2,$B,KP_BLOCK=512" "KP_HASHES=1,$B,KP_BLOCK=512,KP_MIN_WAVES=8" > gpurun_out/r1z/sweep384.log 2>&1
echo "exit=$?"
