#!/bin/bash
# r2q: bench.py step size (nonces per GPU per step): kernel tail and per-step launches vs 2^23 / 2^24 / 2^25.
set -o pipefail
mkdir -p gpurun_out/r2q
for b in 8388608 16777216 33554432 8388608; do
  timeout -k 10 300 python -u bench.py --batch $b --equihash 0 --steps 20 --warmup 3 >> gpurun_out/r2q/bench_batch.jsonl 2>> gpurun_out/r2q/bench.err || exit $?
done
echo "exit=$?"
