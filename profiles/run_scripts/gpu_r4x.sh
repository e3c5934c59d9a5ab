#!/bin/bash
# r4x: resident verify with the header decode beside the device vs before it, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 300 python3 -u tools/verify_overlap_probe.py > $O/overlap.jsonl 2> $O/overlap.err
echo "exit=$?"
