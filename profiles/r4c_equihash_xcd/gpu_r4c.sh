#!/bin/bash
# r4c: Equihash private-slot engine with XCD-local instances (EQP_XCD_LOCAL: every workgroup of an
# instance on one XCD, so one L2 sees all of that instance's row appends) against the default
# mapping, interleaved, at 8 and 16 instances per batch; EA write requests per kernel of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python3 tools/equihash_bench.py --engines ps --batches 12 --variants "" EQP_XCD_LOCAL > $O/eq_xcd8.jsonl 2> $O/eq_xcd8.err &&
timeout -k 10 300 python3 tools/equihash_bench.py --engines ps --inst 16 --batches 8 --variants "" EQP_XCD_LOCAL > $O/eq_xcd16.jsonl 2> $O/eq_xcd16.err &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/pmc_base -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 1 > $O/pmc_base.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/pmc_xcd -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 1 --variants EQP_XCD_LOCAL > $O/pmc_xcd.log 2>&1
echo "exit=$?"
