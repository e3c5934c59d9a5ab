#!/bin/bash
# r4a: KawPow ceiling — the shipping kernel against itself with classes of the period's ops
# compiled out (KP_SKEL_*: gather chain + 11 L1 lookups; gather + math; gather only), same
# occupancy, interleaved rounds; then one LDS/VALU counter pass over the same four variants.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4a
V="tuned tuned+KP_SKEL_NOMATH tuned+KP_SKEL_NOCACHE tuned+KP_SKEL_GATHER"
timeout -k 10 420 python3 -u tools/kawpow_sweep.py --epoch 384 --batch 8388608 --rounds 7 --variants $V \
  --out gpurun_out/r4a/ceiling384.json > gpurun_out/r4a/ceiling384.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/r4a/pmc -o skel -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 \
  --check-windows 0 --variants $V > gpurun_out/r4a/pmc.log 2>&1
echo "exit=$?"
