#!/bin/bash
# r5z2: resident verify after the issue reorder (full hashes before the early copy, the copy at the end of the side stream) and the
# dword-loading SHA-256: verify GPU tests, stage probe, kernel timeline
set -o pipefail
O=gpurun_out/r5z2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_verify.py tests/test_gpu_verify.py tests/test_gpu_sha256.py -v --timeout 200 \
  --timeout-method thread > $O/pytest_verify.log 2>&1 &&
timeout -k 10 200 python3 -u tools/verify_issue_probe.py --runs 30 > $O/issue.json 2> $O/issue.err &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o t --output-format csv \
  -- python3 tools/verify_issue_probe.py --runs 5 > $O/trace.log 2>&1
echo "exit=$?"
