#!/bin/bash
# r4w: the Equihash private-slot engine against its EQP_GLOBAL_SLOTS variant (one global atomic per
# row on the bucket counter, an instance's writers on one XCD so one L2 merges each bucket's tail
# line), interleaved at the mining window's 16 instances; EA write requests per kernel of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 300 python3 tools/equihash_bench.py --engines ps --inst 16 --batches 8 --variants "" EQP_GLOBAL_SLOTS \
  > $O/eq_global16.jsonl 2> $O/eq_global16.err &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/pmc_global -o eq \
  --output-format csv -- python3 tools/equihash_bench.py --engines ps --inst 16 --batches 1 --variants EQP_GLOBAL_SLOTS \
  > $O/pmc_global.log 2>&1
echo "exit=$?"
