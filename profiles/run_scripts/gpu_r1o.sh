#!/bin/bash
# Batch verify stage breakdown + kernel trace of the dense DAG path.
set -o pipefail
mkdir -p gpurun_out/r1o
timeout -k 10 300 python -u tools/verify_bench.py --cpu-sample 4 --modes dag light > gpurun_out/r1o/verify_bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r1o/prof -o verify -- python3 tools/verify_bench.py --cpu-sample 1 --modes dag > gpurun_out/r1o/prof.log 2>&1
