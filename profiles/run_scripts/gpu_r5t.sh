#!/bin/bash
# r5t: a fresh box's build_all (must keep the shipped libraries), the resident verify's host parts
# (materialize / prepare / commit on their own) and the X16R per-slot step latency
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python3 -c "import os, time; from nodexa_chain_core_amd import _build as b; so = os.path.join(b.PKG, '_core' + b.EXT); m = os.stat(so).st_mtime_ns; t = time.time(); b.build_all(); print('build_all', round(time.time() - t, 2), 's, _core kept' if os.stat(so).st_mtime_ns == m else 's, _core REBUILT')" > $O/build.log 2>&1 &&
timeout -k 10 200 python3 -u tools/verify_issue_probe.py --runs 30 > $O/issue.json 2> $O/issue.err &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 16384 > gpurun_out/r5t/slots16k.json 2> gpurun_out/r5t/slots.err &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 65536 > gpurun_out/r5t/slots65k.json 2>> gpurun_out/r5t/slots.err
echo "exit=$?"
