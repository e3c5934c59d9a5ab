#!/bin/bash
# r4q: calibrate TCC_EA0_WRREQ against a known store pattern (tools/scatter_ceiling.hip: 64M random
# rows per launch of 16..64 bytes, and G-lane runs), so the Equihash rounds' "2.0-2.5 EA write
# requests per row" (r4c / r4l) can be read as requests per row or as a counter convention.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4q
mkdir -p $O
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/scatter -o s \
  --output-format csv -- tools/bin/scatter_ceiling > $O/scatter.log 2>&1 || exit $?
echo "exit=0"
