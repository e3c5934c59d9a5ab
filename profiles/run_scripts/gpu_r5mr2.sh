#!/bin/bash
# r5mr2: the two-rank GPU test with the verify part
set -o pipefail
O=gpurun_out/r5mr2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multirank.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "exit=$?"
