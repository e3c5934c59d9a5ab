#!/bin/bash
# (KP_PF_MAX was removed in round 5 after this A/B: it lost; the code is at commit 65a1eaa)
# r5d: KawPow cross-round lookahead (KP_PF_MAX: the first N cache ops whose source register is final
# when the previous round's program ends read the L1 under that round's DAG wait), interleaved A/B,
# every variant bit-exact over its share windows; the collective-stream dispatch probe while two
# search windows are resident; then the Equihash geometries (r5c).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 500 python3 -u tools/kawpow_sweep.py --epoch 384 --batch 8388608 --rounds 7 \
  --variants tuned tuned+KP_PF_MAX=2 tuned+KP_PF_MAX=4 tuned+KP_PF_MAX=8 --out $O/pf384.json > $O/pf384.log 2>&1 &&
timeout -k 10 200 python3 -u tools/coll_dispatch_probe.py --epoch 384 --windows 6 > $O/dispatch.json 2> $O/dispatch.err &&
tools/gpu_r5c.sh
