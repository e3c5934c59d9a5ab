#!/bin/bash
# r3zh: round-3 final tree — GPU tier + smoke + bench (tools/gpu_rehearsal.sh), then a
# rocprofv3 kernel-trace/stats pass over a short bench run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
bash tools/gpu_rehearsal.sh r3zh &&
grep -q '"metric"' gpurun_out/r3zh/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3zh/prof -o bench \
  -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/r3zh/prof_bench.log 2>&1
echo "exit=$?"
