#!/bin/bash
# GPU tier + smoke + driver-contract bench into gpurun_out/<tag>/ (usage: tools/gpu_rehearsal.sh <tag>)
set -o pipefail
tag=${1:?tag}
mkdir -p gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/$tag/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
echo "exit=$?"
