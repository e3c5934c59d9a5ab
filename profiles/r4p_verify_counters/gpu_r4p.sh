#!/bin/bash
# r4p: counters of the two full-hash verify kernels on the 10k-header bench batch: the LDS-mix
# interpreter (kawpow_verify_dag, NODEXA_VERIFY_WAVES=0) and the wave-uniform one
# (kawpow_verify_waves): instruction mix, LDS traffic, waits.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4p
mkdir -p $O
C="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES"
NODEXA_VERIFY_WAVES=0 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C -d $O/dag -o v --output-format csv \
  -- python3 bench.py --steps 1 --warmup 0 --equihash 0 --verify 1 --check-shares 1 > $O/dag.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C -d $O/waves -o v --output-format csv \
  -- python3 bench.py --steps 1 --warmup 0 --equihash 0 --verify 1 --check-shares 1 > $O/waves.log 2>&1 || exit $?
echo "exit=0"
