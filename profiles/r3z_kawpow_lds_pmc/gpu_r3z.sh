#!/bin/bash
# r3z: LDS vs VALU vs memory-wait counters of the default KawPow kernel (backs the LDS-bound reading
# of profiles/README r3v/r3w): LDS-array active cycles and bank-conflict cycles, LDS / VALU issue
# activity and instruction waits, against GRBM_GUI_ACTIVE.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3z
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r3z -o lds -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/r3z/pmc_lds.log 2>&1
echo "exit=$?"
