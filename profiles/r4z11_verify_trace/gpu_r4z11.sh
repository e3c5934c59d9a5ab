#!/bin/bash
# r4z11: kernel + memory-copy trace of the resident verify (the early hashes + nBits copy beside the
# full-hash kernels), from the overlap probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4z11
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o v --output-format csv \
  -- python3 tools/verify_overlap_probe.py > $O/trace.log 2>&1
echo "exit=$?"
