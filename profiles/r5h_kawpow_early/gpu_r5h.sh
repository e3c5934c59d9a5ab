#!/bin/bash
# (KP_EARLY was removed after this A/B: it lost; the code is at commit 65a1eaa)
# r5h: KawPow in-round early issue (KP_EARLY=N: the first N L1 lookups whose source register no
# earlier op of the round writes are issued together as the round's first LDS reads; the ISA goes
# from 11 serialized ds_read -> s_waitcnt lgkmcnt(0) pairs to one batch plus the dependent ones),
# interleaved A/B, every variant bit-exact over its share windows, at two epochs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 560 python3 -u tools/kawpow_sweep.py --epoch 384 --batch 8388608 --rounds 7 \
  --variants tuned tuned+KP_EARLY=3 tuned+KP_EARLY=6 tuned+KP_EARLY=11 tuned+KP_EARLY=11+KP_EARLY_FENCE \
  --out $O/early384.json > $O/early384.log 2>&1 &&
timeout -k 10 400 python3 -u tools/kawpow_sweep.py --epoch 100 --batch 8388608 --rounds 5 \
  --variants tuned tuned+KP_EARLY=6 tuned+KP_EARLY=11 --out $O/early100.json > $O/early100.log 2>&1
