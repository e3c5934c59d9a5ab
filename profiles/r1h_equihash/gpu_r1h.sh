#!/bin/bash
# (1) Equihash round-kernel variants (compact LDS rows, batched slot atomics) + GPU Equihash tests;
# (2) mixed KawPow+Equihash synthetic chain (BASELINE config 5) and its batch-verify bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1h gpurun_out/data
timeout -k 10 200 python -u -m pytest tests/test_gpu_equihash.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r1h/pytest_eq.log 2>&1 && \
timeout -k 10 300 python -u tools/equihash_bench.py --inst 8 --batches 8 --variants "" EQ_COMPACT_LDS EQ_EMIT_BATCH=2 EQ_EMIT_BATCH=4 "EQ_COMPACT_LDS,EQ_EMIT_BATCH=2" "EQ_COMPACT_LDS,EQ_EMIT_BATCH=4" > gpurun_out/r1h/eq_variants.log 2>&1 && \
timeout -k 10 600 python -u tools/make_synthetic_chain.py --n 9830 --equihash 170 --backend gpu --out gpurun_out/data/testnet_mixed_10k.hdr > gpurun_out/r1h/mine_mixed.log 2>&1 && \
timeout -k 10 200 python -u tools/verify_bench.py --file gpurun_out/data/testnet_mixed_10k.hdr --cpu-sample 10 > gpurun_out/r1h/verify_bench_mixed.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
