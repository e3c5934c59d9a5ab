#!/bin/bash
# r4v: Equihash-shaped append probes (tools/scatter_ceiling.hip "a" mode): private slot segments
# (the shipping scheme) against one global atomic per row on the bucket counter with an instance's
# writers on one XCD, so that the L2 merges a bucket's rows; times and EA write requests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 60 tools/bin/scatter_ceiling a > $O/append.jsonl 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum -d $O/pmc -o a \
  --output-format csv -- tools/bin/scatter_ceiling a > $O/pmc.log 2>&1 || exit $?
echo "exit=0"
