#!/bin/bash
# Round-1 second GPU pass: GPU tests, smoke, bench, then rocprofv3 kernel stats and SQ/LDS
# counters of the tuned KawPow search (counters in their own --kernel-trace runs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof2 gpurun_out/pmc2
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o bench -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof2_bench.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc2 -o sq -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/pmc2_sq.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc2 -o lds -- python3 tools/kawpow_sweep.py --rounds 1 --batch 4194304 > gpurun_out/pmc2_lds.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
