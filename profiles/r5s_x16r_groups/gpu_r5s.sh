#!/bin/bash
# r5s: X16R batch with the native slot grouping (_core.x16r_groups): GPU X16R tests and the probe
set -o pipefail
O=gpurun_out/r5s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_x16r.py -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u tools/x16r_probe.py --n 65536 --reps 3 > $O/probe.json 2> $O/probe.err &&
timeout -k 10 300 python3 -u tools/x16r_probe.py --n 16384 --reps 3 > $O/probe16k.json 2> $O/probe16k.err
echo "exit=$?"
