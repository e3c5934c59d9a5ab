#!/bin/bash
# r3za: rehearsal of the N>1 bench path on the 1-GPU box: two torchrun ranks share GPU 0 and
# exchange over gloo (RCCL refuses two ranks on one device), so the sharded DAG build + all-gather,
# the mining loop's packet broadcast / share gather, the MAX-over-ranks timing and the rank-0 JSON
# line all run as they do at N=2 on a node (hash rate is the one GPU's, split two ways).
set -o pipefail
mkdir -p gpurun_out/r3za
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
NODEXA_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 2 --steps 6 --warmup 2 \
  > gpurun_out/r3za/bench2.json 2> gpurun_out/r3za/bench2.err
echo "exit=$?"
