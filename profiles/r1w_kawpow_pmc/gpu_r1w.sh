#!/bin/bash
# PMC pass over the current tuned KawPow search (KP_SBUFFER): VALU / LDS per hash, bank conflicts, L2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1w
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/r1w -o sq -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/r1w/pmc_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r1w -o lds -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/r1w/pmc_lds.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/r1w -o tcc -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/r1w/pmc_tcc.log 2>&1
echo "exit=$?"
