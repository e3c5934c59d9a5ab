#!/bin/bash
# r5g: kawpow_verify_waves with branch-free op selection (KW_SELECT): bit-exactness against the LDS
# interpreter and the host golden model (GPU tests), the verify pipeline's kernel stats, and the
# bench line with the corrected device-clock rate.
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_verify.py tests/test_gpu_verify.py -v --timeout 200 \
  --timeout-method thread > $O/pytest_verify.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_verify -o v --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --equihash 0 --verify 1 > $O/prof_verify.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo "exit=$?"
