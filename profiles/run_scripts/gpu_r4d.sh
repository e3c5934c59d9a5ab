#!/bin/bash
# r4d: why the node's Equihash windows (16 instances) run at ~2 Sol/s in bench.py while the
# 8-instance standalone solver runs at ~3k: per-instance solutions vs the golden solver, host
# re-solves and collect times at 8 and 16 instances.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 400 python3 -u tools/eq_window_probe.py > $O/probe.jsonl 2> $O/probe.err
echo "exit=$?"
