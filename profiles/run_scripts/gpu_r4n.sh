#!/bin/bash
# r4n: the staged DAG verify path (verifyheaders RPC / process_headers "dag") on kawpow_verify_waves.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_verify.py \
  tests/test_gpu_mixonly.py > $O/pytest.log 2>&1 || exit $?
echo "exit=0"
