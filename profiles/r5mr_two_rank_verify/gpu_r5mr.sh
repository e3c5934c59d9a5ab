#!/bin/bash
# r5mr: the N>1 bench with the verify part (resident pipeline sliced over 2 ranks + all-gather),
# two torchrun ranks on GPU 0 over gloo (RCCL refuses two ranks on one device)
set -o pipefail
O=gpurun_out/r5mr
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
NODEXA_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 8388608 \
  --equihash 0 --verify 1 --check-shares 2 > $O/bench2.json 2> $O/bench2.err
echo "exit=$?"
