#!/bin/bash
# r4t: does the L2 merge rows that different store instructions write into one line (same-XCD vs
# all-XCD sharing), and what do random row gathers cost (tools/scatter_ceiling.hip "m" mode).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 60 tools/bin/scatter_ceiling m > $O/merge.jsonl 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum -d $O/pmc -o m \
  --output-format csv -- tools/bin/scatter_ceiling m > $O/pmc.log 2>&1 || exit $?
echo "exit=0"
