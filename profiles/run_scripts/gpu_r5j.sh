#!/bin/bash
# r5j: classic Ethash on the GPU after the split into seed / mix / final kernels: bit-exactness of
# batch hashes and of the device-side search against the host golden model; shipped throughput.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kawpow.py -x -v --timeout 240 --timeout-method thread \
  -k "hashimoto or ethash_search or dag_l1" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u tools/hashimoto_probe.py --epoch 384 --jobs 4194304 --reps 7 > $O/probe384.json 2> $O/probe384.err
