#!/bin/bash
# r2b: KP_NT_DAG on the large-DAG pointer path (epoch 390, DAG > 4 GiB) and KP_MUL33_SHIFT at 384.
set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 420 python -u tools/kawpow_sweep.py --epoch 390 --rounds 7 --variants tuned tuned-KP_NT_DAG \
  > gpurun_out/r2b/sweep390.log 2>&1 &&
timeout -k 10 420 python -u tools/kawpow_sweep.py --epoch 384 --rounds 7 --variants tuned tuned+KP_MUL33_SHIFT \
  > gpurun_out/r2b/sweep384.log 2>&1
echo "exit=$?"
