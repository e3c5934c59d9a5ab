#!/bin/bash
# Equihash: refs carried in the row slot (one scattered write per row) vs separate refs, x compact LDS.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1k
timeout -k 10 200 python -u -m pytest tests/test_gpu_equihash.py tests/test_gpu_verify.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r1k/pytest_eq.log 2>&1 && \
timeout -k 10 300 python -u tools/equihash_bench.py --inst 8 --batches 8 --variants "" EQ_SEPARATE_REFS EQ_COMPACT_LDS "EQ_SEPARATE_REFS,EQ_COMPACT_LDS" > gpurun_out/r1k/eq_variants.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/r1k/pmc -o tcc -- python3 tools/equihash_bench.py --inst 8 --batches 1 > gpurun_out/r1k/pmc_tcc.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
