#!/bin/bash
# r5c: coarse-bucket Equihash: exactness of the two-phase staging (tests), then geometries (D = 256 /
# 512 / 1024 coarse buckets = slices per bucket 4 / 2 / 1) and producer shapes against the
# private-slot engine, interleaved, 16 instances per batch; kernel stats of the best candidates.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_equihash.py -v --timeout 120 --timeout-method thread \
  > $O/pytest_eq.log 2>&1
rc=$?; [ $rc -le 1 ] || { echo "pytest rc=$rc: stop"; exit $rc; }
timeout -k 10 400 python3 -u tools/equihash_bench.py --inst 16 --batches 6 --engines cb --variants "" \
  "EQC_COARSE_BITS=9,EQC_KMAX=12" "EQC_COARSE_BITS=10,EQC_KMAX=6" "EQC_B2=2" \
  > $O/eq16_cb.jsonl 2> $O/eq16_cb.err &&
timeout -k 10 200 python3 -u tools/equihash_bench.py --inst 16 --batches 6 --engines ps > $O/eq16_ps.jsonl 2> $O/eq16_ps.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o eq --output-format csv \
  -- python3 tools/equihash_bench.py --inst 16 --batches 3 --engines cb > $O/prof.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof10 -o eq --output-format csv \
  -- python3 tools/equihash_bench.py --inst 16 --batches 3 --engines cb --variants "EQC_COARSE_BITS=10,EQC_KMAX=6" > $O/prof10.log 2>&1
echo "exit=$?"
