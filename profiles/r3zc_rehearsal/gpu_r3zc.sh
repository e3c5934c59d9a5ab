#!/bin/bash
# r3zc: GPU tier + smoke + bench after the Equihash candidate/chain cap change (kernel_params.h is
# part of the KawPow template digest, so the period kernels were rebuilt too).
set -o pipefail
mkdir -p gpurun_out/r3zc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3zc/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3zc/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3zc/bench.json 2> gpurun_out/r3zc/bench.err
echo "exit=$?"
