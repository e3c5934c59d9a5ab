#!/bin/bash
# r4m: producer threads per round workgroup (EQP_NP; 448 = 7 of 16 waves, r3's best at P=32 / 8
# instances) re-swept in the new shape: P=16, 16 instances, final round 256 wide.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 500 python3 tools/equihash_bench.py --inst 16 --batches 10 --engines ps:16:1024:256 \
  --variants "" EQP_NP=384 EQP_NP=512 EQP_NP=576 > $O/eq_np.jsonl 2> $O/eq_np.err || exit $?
echo "exit=0"
