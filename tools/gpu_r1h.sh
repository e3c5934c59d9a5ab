#!/bin/bash
# Mixed KawPow+Equihash synthetic chain (BASELINE config 5) and its batch-verify bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1h gpurun_out/data
timeout -k 10 900 python -u tools/make_synthetic_chain.py --n 9830 --equihash 170 --backend gpu --out gpurun_out/data/testnet_mixed_10k.hdr > gpurun_out/r1h/mine_mixed.log 2>&1 && \
timeout -k 10 200 python -u tools/verify_bench.py --file gpurun_out/data/testnet_mixed_10k.hdr --cpu-sample 10 > gpurun_out/r1h/verify_bench_mixed.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
