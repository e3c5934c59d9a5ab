#!/bin/bash
# r4s: the resident verify GPU tests including the shared miner DAG test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_resident_verify.py \
  > $O/pytest.log 2>&1 || exit $?
echo "exit=0"
