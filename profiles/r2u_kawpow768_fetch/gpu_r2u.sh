#!/bin/bash
# r2u: HBM traffic of the 768-thread KawPow default (FETCH_SIZE alone: 3 of the 4 TCC counters).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2u
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2u -o tcc -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/r2u/pmc_tcc.log 2>&1
echo "exit=$?"
