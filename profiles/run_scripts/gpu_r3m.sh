#!/bin/bash
# r3m: Equihash PS dense pair-list emission: exactness, device time, per-kernel time, store counts.
set -o pipefail
mkdir -p gpurun_out/r3m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_equihash.py -v --timeout 200 -k "ps" > gpurun_out/r3m/pytest_eq.log 2>&1 &&
timeout -k 10 200 python -u tools/equihash_bench.py --engines ps --batches 8 --inst 8 > gpurun_out/r3m/eb8.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3m/prof -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 4 > gpurun_out/r3m/prof.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d gpurun_out/r3m/p4 -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 1 > gpurun_out/r3m/p4.log 2>&1
echo "exit=$?"
