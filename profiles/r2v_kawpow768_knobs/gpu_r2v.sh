#!/bin/bash
# r2v: cache-policy and modulo knobs re-checked on the 768-thread default (epoch 384).
set -o pipefail
mkdir -p gpurun_out/r2v
timeout -k 10 600 python -u tools/kawpow_sweep.py --epoch 384 --rounds 7 --out gpurun_out/r2v/sweep384.jsonl \
  --variants tuned tuned-KP_NT_DAG tuned+KP_FASTMOD24 > gpurun_out/r2v/sweep384.log 2>&1
echo "exit=$?"
