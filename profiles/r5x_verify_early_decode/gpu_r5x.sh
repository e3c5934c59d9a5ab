#!/bin/bash
# r5x: the resident verify with the header decode started before the issue stage (helper thread)
set -o pipefail
O=gpurun_out/r5x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_verify.py tests/test_gpu_verify.py -v --timeout 200 \
  --timeout-method thread > $O/pytest_verify.log 2>&1 &&
timeout -k 10 200 python3 -u tools/verify_issue_probe.py --runs 30 > $O/issue.json 2> $O/issue.err &&
NODEXA_VERIFY_OVERLAP=0 timeout -k 10 200 python3 -u tools/verify_issue_probe.py --runs 30 > $O/issue_nooverlap.json 2> $O/issue2.err
echo "exit=$?"
