#!/bin/bash
# r5o: kawpow_verify_waves round cost breakdown (tools/verify_waves_variants.hip, prebuilt here to
# tools/pv_waves.hsaco) and rocprof stats of the replay.
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 120 python3 -u tools/verify_waves_probe.py --hsaco tools/pv_waves.hsaco --variants 9 10 > $O/probe.json 2> $O/probe.err
echo "exit=$?"
