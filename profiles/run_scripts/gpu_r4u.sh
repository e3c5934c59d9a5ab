#!/bin/bash
# r4u: batch verify with the header objects decoded beside the device (HeaderBatch deferred
# decode): the resident-verify GPU tests, then the driver-contract bench line.
set -o pipefail
mkdir -p gpurun_out/r4u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_verify.py tests/test_gpu_verify.py -v --timeout 240 \
  --timeout-method thread > gpurun_out/r4u/pytest.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r4u/bench.json 2> gpurun_out/r4u/bench.err
echo "exit=$?"
