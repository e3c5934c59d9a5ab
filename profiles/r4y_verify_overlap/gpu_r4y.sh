#!/bin/bash
# r4y: the driver-contract bench line with the verify runs' chains made right before each run
# (median of 15), and the overlap A/B probe again on the same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4y
mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python3 -u tools/verify_overlap_probe.py > $O/overlap.jsonl 2> $O/overlap.err
echo "exit=$?"
