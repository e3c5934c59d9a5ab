#!/bin/bash
# Equihash round-kernel variants (compact LDS rows, batched slot atomics) + GPU Equihash tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1i
timeout -k 10 200 python -u -m pytest tests/test_gpu_equihash.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r1i/pytest_eq.log 2>&1 && \
timeout -k 10 300 python -u tools/equihash_bench.py --inst 8 --batches 8 --variants "" EQ_COMPACT_LDS EQ_EMIT_BATCH=2 EQ_EMIT_BATCH=4 "EQ_COMPACT_LDS,EQ_EMIT_BATCH=2" "EQ_COMPACT_LDS,EQ_EMIT_BATCH=4" > gpurun_out/r1i/eq_variants.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
