#!/bin/bash
# r5z: kernel + memory-copy timeline of the resident verify (which stream waits on which)
set -o pipefail
O=gpurun_out/r5z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o t --output-format csv \
  -- python3 tools/verify_issue_probe.py --runs 5 > $O/trace.log 2>&1
echo "exit=$?"
