#!/bin/bash
# r3zg: KP_L1G — some of each round's 11 L1 lookups read the DAG's first 16 KiB through the vector
# L1 (buffer_load) instead of the LDS copy, against the LDS-only default (profiles/r3z: LDS ~74 % busy).
set -o pipefail
mkdir -p gpurun_out/r3zg
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 600 python -u tools/kawpow_sweep.py --rounds 7 --variants tuned \
  tuned+KP_L1G=1 tuned+KP_L1G=3 tuned+KP_L1G=33 tuned+KP_L1G=7 tuned+KP_L1G=585 tuned+KP_L1G=1024 tuned+KP_L1G=2047 \
  --out gpurun_out/r3zg/sweep384.json > gpurun_out/r3zg/sweep384.log 2>&1
echo "exit=$?"
