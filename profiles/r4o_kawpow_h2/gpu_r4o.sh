#!/bin/bash
# r4o: two interleaved hash chains per 16-lane group (KP_HASHES=2: more independent work per wave to
# cover the conflicted L1 lookups) at 512 threads / 4 waves per SIMD (128 VGPRs), against the
# shipping 768-thread single-chain kernel; epoch 384, interleaved rounds, bit-exactness checked.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 500 python3 -u tools/kawpow_sweep.py --epoch 384 --batch 8388608 --rounds 7 --variants tuned \
  "tuned-KP_HASHES=1+KP_HASHES=2-KP_BLOCK=768-KP_MIN_WAVES=6+KP_BLOCK=512+KP_MIN_WAVES=4" \
  --out $O/sweep_h2.json > $O/sweep_h2.log 2>&1 || exit $?
echo "exit=0"
