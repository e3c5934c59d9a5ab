#!/bin/bash
# r5t: the resident verify's host parts (materialize / prepare / commit on their own)
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 200 python3 -u tools/verify_issue_probe.py --runs 30 > $O/issue.json 2> $O/issue.err
echo "exit=$?"
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 16384 > gpurun_out/r5t/slots16k.json 2> gpurun_out/r5t/slots.err &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 65536 > gpurun_out/r5t/slots65k.json 2>> gpurun_out/r5t/slots.err
echo "exit2=$?"
