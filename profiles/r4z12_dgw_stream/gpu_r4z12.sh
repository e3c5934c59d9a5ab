#!/bin/bash
# r4z12: DGW on its own stream beside the Equihash checks: verify GPU tests, a kernel + copy trace
# of the probe, the overlap A/B probe and the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4z12
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_verify.py tests/test_gpu_verify.py -v --timeout 240 \
  --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o v --output-format csv \
  -- python3 tools/verify_overlap_probe.py > $O/trace.log 2>&1 &&
timeout -k 10 300 python3 -u tools/verify_overlap_probe.py > $O/overlap.jsonl 2> $O/overlap.err &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo "exit=$?"
