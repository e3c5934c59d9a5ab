#!/bin/bash
# r5u: SIMD-512 with the final block's constant expansion and the sparse first NTT stages: GPU X16R tests, per-slot step latency, batch probe
set -o pipefail
O=gpurun_out/r5u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_x16r.py -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 16384 > $O/slots16k.json 2> $O/slots.err &&
timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 65536 > $O/slots65k.json 2>> $O/slots.err &&
timeout -k 10 300 python3 -u tools/x16r_probe.py --n 65536 --reps 3 > $O/probe.json 2> $O/probe.err &&
timeout -k 10 300 python3 -u tools/x16r_probe.py --n 16384 --reps 3 > $O/probe16k.json 2> $O/probe16k.err
echo "exit=$?"
