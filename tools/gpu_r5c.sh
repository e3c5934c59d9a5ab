#!/bin/bash
# r5c: coarse-bucket Equihash geometries (D = 256 / 512 / 1024 coarse buckets = re-read factor 4 / 2 /
# 1) and producer shapes against the private-slot engine, interleaved, 16 instances per batch.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 400 python3 -u tools/equihash_bench.py --inst 16 --batches 6 --engines cb --variants "" \
  "EQC_COARSE_BITS=9,EQC_SLICE_BITS=1" "EQC_COARSE_BITS=10,EQC_SLICE_BITS=0" "EQC_BATCH=4" "EQC_NP=640" \
  > $O/eq16_cb.jsonl 2> $O/eq16_cb.err &&
timeout -k 10 200 python3 -u tools/equihash_bench.py --inst 16 --batches 6 --engines ps > $O/eq16_ps.jsonl 2> $O/eq16_ps.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof10 -o eq --output-format csv \
  -- python3 tools/equihash_bench.py --inst 16 --batches 3 --engines cb --variants "EQC_COARSE_BITS=10,EQC_SLICE_BITS=0" > $O/prof10.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof9 -o eq --output-format csv \
  -- python3 tools/equihash_bench.py --inst 16 --batches 3 --engines cb --variants "EQC_COARSE_BITS=9,EQC_SLICE_BITS=1" > $O/prof9.log 2>&1
echo "exit=$?"
