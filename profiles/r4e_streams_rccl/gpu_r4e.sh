#!/bin/bash
# r4e: (0) the KawPow GPU tests; (1) bench.py with Equihash through the node loop on the GPU solver (the bare-device routing
# fix); (2) the one-rank RCCL bench with the collectives on high-priority streams, against the
# plain run; (3) a kernel trace of the RCCL run: the collectives' copies must run while the next
# search window is queued, not after it (queue ids per dispatch).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e
mkdir -p $O
# the search kernel without the LDS-digest form: bit-exact at epochs 384 (768 threads) and 390
# (pointer path, 512 threads, digests in registers)
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_kawpow.py \
  > $O/pytest_kawpow.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --collectives > $O/bench_rccl.json 2> $O/bench_rccl.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o rccl \
  -- python3 bench.py --steps 6 --warmup 2 --collectives --verify 0 --equihash 4 > $O/prof_rccl.log 2>&1
echo "exit=$?"
