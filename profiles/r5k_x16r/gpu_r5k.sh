#!/bin/bash
# r5k: X16R / X16RV2 on the GPU (x16r.hip): chain vectors + host equivalence, throughput, kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_x16r.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u tools/x16r_probe.py --n 65536 --reps 3 > $O/probe.json 2> $O/probe.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o x --output-format csv -- python3 tools/x16r_probe.py --n 16384 --reps 1 > $O/probe_prof.json 2> $O/probe_prof.err
