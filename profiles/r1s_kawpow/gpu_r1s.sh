#!/bin/bash
# KawPow DAG addressing: raw buffer (KP_BUFFER, < 4 GiB) vs structured buffer (KP_SBUFFER, any size)
# at epoch 384, and the > 4 GiB case (epoch 390): 64-bit pointers (old fallback) vs KP_SBUFFER.
set -o pipefail
mkdir -p gpurun_out/r1s
T="KP_HASHES=1,KP_DPP,KP_BARRETT,KP_L1X4,KP_BLOCK=512"
timeout -k 10 300 python -u tools/kawpow_sweep.py --epoch 384 --rounds 7 --variants tuned "$T,KP_SBUFFER" > gpurun_out/r1s/sweep384.log 2>&1 &&
timeout -k 10 300 python -u tools/kawpow_sweep.py --epoch 390 --rounds 7 --variants "$T" "$T,KP_SBUFFER" > gpurun_out/r1s/sweep390.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kawpow.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r1s/pytest_kawpow.log 2>&1
