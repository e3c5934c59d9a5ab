#!/bin/bash
# r4j: P2P header sync through the resident path, native wave slot tables, Equihash back on one
# solver per device: GPU tests, then the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_resident_verify.py \
  tests/test_gpu_equihash_mining.py tests/test_gpu_rccl.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "exit=0"
