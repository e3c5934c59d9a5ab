#!/bin/bash
# r4k: Equihash private-slot engine writers per instance (P) at the mining window's 16 instances:
# P=16 is one 1024-thread workgroup per CU for the whole round (256 workgroups), P=32 two rounds
# of workgroups, P=64 four; and the final round's width (1024 workgroups per instance by default,
# 256 / 64); interleaved device times per batch.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 400 python3 tools/equihash_bench.py --inst 16 --batches 10 \
  --engines ps:16 ps:32 ps:64 ps:32:1024:256 ps:32:1024:64 ps:16:1024:256 \
  > $O/eq_groups16.jsonl 2> $O/eq_groups16.err || exit $?
timeout -k 10 400 python3 tools/equihash_bench.py --inst 8 --batches 10 --engines ps:16 ps:32 \
  > $O/eq_groups8.jsonl 2> $O/eq_groups8.err || exit $?
echo "exit=0"
