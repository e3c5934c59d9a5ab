#!/bin/bash
# Equihash round kernels under rocprofv3: kernel stats, then SQ and TCC counters in separate passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1j
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1j/stats -o eq -- python3 tools/equihash_bench.py --inst 8 --batches 3 > gpurun_out/r1j/stats.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/r1j/pmc -o sq -- python3 tools/equihash_bench.py --inst 8 --batches 1 > gpurun_out/r1j/pmc_sq.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/r1j/pmc -o tcc -- python3 tools/equihash_bench.py --inst 8 --batches 1 > gpurun_out/r1j/pmc_tcc.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r1j/pmc -o lds -- python3 tools/equihash_bench.py --inst 8 --batches 1 > gpurun_out/r1j/pmc_lds.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
