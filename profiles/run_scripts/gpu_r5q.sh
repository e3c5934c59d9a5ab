#!/bin/bash
# r5q: kawpow_verify_waves with the handler-table dispatch: verify GPU tests (bit-exactness against
# the LDS interpreter and the host), the kernel against the branch-tree build (probe variant 0),
# the resident pipeline's stage times and the verify kernel stats.
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_verify.py tests/test_gpu_verify.py -v --timeout 200 \
  --timeout-method thread > $O/pytest_verify.log 2>&1 &&
timeout -k 10 120 python3 -u tools/verify_waves_probe.py --hsaco tools/pv_waves.hsaco --variants 0 9 > $O/probe.json 2> $O/probe.err &&
timeout -k 10 200 python3 -u tools/verify_issue_probe.py --runs 30 > $O/issue.json 2> $O/issue.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_verify -o v --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --equihash 0 --verify 1 > $O/prof_verify.log 2>&1
echo "exit=$?"
