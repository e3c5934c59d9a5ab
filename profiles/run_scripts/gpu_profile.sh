#!/bin/bash
# Profiling pass on one MI355X: kernel trace + stats, PMC counters (separate run),
# and an in-process A/B sweep of search-kernel variants. Output under gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof gpurun_out/pmc
timeout -k 10 200 python tools/kawpow_sweep.py --rounds 5 --variants "" "KP_NT_DAG" "KP_MIN_WAVES=6" > gpurun_out/sweep.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_bench.log 2>&1 && \
(rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true) && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc -o sq -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/pmc_sq.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc -o tcc -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/pmc_tcc.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc -o lds -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/pmc_lds.log 2>&1
echo "exit=$?"
