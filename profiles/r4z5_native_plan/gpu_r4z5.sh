#!/bin/bash
# r4z5: native batch plan (ranges, heights, times, bits in one pass) on top of r4z4's two-phase insert (early
# hashes + nBits copy, commit after the verdicts): the verify GPU tests, the overlap A/B probe and
# the driver-contract bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4z5
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_verify.py tests/test_gpu_verify.py -v --timeout 240 \
  --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u tools/verify_overlap_probe.py > $O/overlap.jsonl 2> $O/overlap.err &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo "exit=$?"
