#!/bin/bash
# Equihash: current default (refs in slot, compact LDS, alignbit rotates) vs LDS stride-5 padding vs full LDS rows.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1m
timeout -k 10 200 python -u -m pytest tests/test_gpu_equihash.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r1m/pytest_eq.log 2>&1 && \
timeout -k 10 300 python -u tools/equihash_bench.py --inst 8 --batches 10 --variants "" EQ_LDS_PAD5 EQ_FULL_LDS > gpurun_out/r1m/eq_variants.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
