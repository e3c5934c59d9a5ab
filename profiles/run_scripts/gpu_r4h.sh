#!/bin/bash
# r4h: resident verify with the side-stream / concurrent-epoch schedule (GPU tests + bench line +
# kernel trace), the two-rank bench on one GPU, and smoke().
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_resident_verify.py \
  tests/test_gpu_verify.py tests/test_gpu_multirank.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_verify -o v \
  -- python3 bench.py --steps 2 --warmup 1 --equihash 0 --verify 1 > $O/prof_verify.log 2>&1 || exit $?
echo "exit=0"
