#!/bin/bash
# r3l: Equihash PS counters per kernel: HBM-side bytes (FETCH_SIZE / WRITE_SIZE), request
# counts, LDS and VALU instruction mix.
set -o pipefail
mkdir -p gpurun_out/r3l
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/r3l/p1 -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 1 > gpurun_out/r3l/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/r3l/p2 -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 1 > gpurun_out/r3l/p2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/r3l/p3 -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 1 > gpurun_out/r3l/p3.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d gpurun_out/r3l/p4 -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 1 > gpurun_out/r3l/p4.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE -d gpurun_out/r3l/p5 -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 1 > gpurun_out/r3l/p5.log 2>&1
echo "exit=$?"
