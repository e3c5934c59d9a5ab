#!/bin/bash
# r5y: the driver-contract bench line after naming the verify modes
set -o pipefail
O=gpurun_out/r5y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo "exit=$?"
