#!/bin/bash
# KawPow item-index modulo: 32-bit Barrett (tuned) vs 24-bit Barrett (KP_FASTMOD24) at epoch 384,
# then the GPU KawPow tests with the 24-bit variant selected.
set -o pipefail
mkdir -p gpurun_out/r1x
T="KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=512"
timeout -k 10 300 python -u tools/kawpow_sweep.py --epoch 384 --rounds 7 --variants tuned "$T,KP_FASTMOD24" > gpurun_out/r1x/sweep384.log 2>&1 &&
NODEXA_KAWPOW_DEFINES="$T,KP_FASTMOD24" timeout -k 10 300 python -u -m pytest tests/test_gpu_kawpow.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r1x/pytest_kawpow24.log 2>&1
echo "exit=$?"
