#!/bin/bash
# r5i: classic Ethash hashimoto on the GPU (ethash_hashimoto.hip) -- bit-exactness against the host
# golden model, throughput at epoch 384 for 1 / 2 / 4 / 8 hashes per 16-lane row, kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kawpow.py -x -v --timeout 240 --timeout-method thread \
  -k "hashimoto or dag_l1" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u tools/hashimoto_probe.py --epoch 384 --jobs 4194304 --reps 5 \
  --kernels ethash_mix_batch_h1 ethash_mix_batch_h2 ethash_mix_batch ethash_mix_batch_h8 > $O/probe384.json 2> $O/probe384.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o hp --output-format csv -- python3 tools/hashimoto_probe.py --epoch 100 --jobs 4194304 --reps 3 > $O/probe100.json 2> $O/probe100.err
