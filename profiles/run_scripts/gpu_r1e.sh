#!/bin/bash
# Mine the BASELINE config-5 synthetic chains on the GPU (fixtures), then the batch-verify bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1e gpurun_out/data
timeout -k 10 100 python -u tools/scan_timing.py 32768 > gpurun_out/r1e/scan32k.log 2>&1 && \
timeout -k 10 400 python -u tools/make_synthetic_chain.py --n 10000 --backend gpu --out gpurun_out/data/testnet_kawpow_10k.hdr > gpurun_out/r1e/mine_kawpow.log 2>&1 && \
timeout -k 10 300 python -u tools/verify_bench.py --file gpurun_out/data/testnet_kawpow_10k.hdr --cpu-sample 20 > gpurun_out/r1e/verify_bench.log 2>&1 && \
timeout -k 10 300 python -u tools/make_synthetic_chain.py --n 9000 --equihash 1000 --backend gpu --out gpurun_out/data/testnet_mixed_10k.hdr > gpurun_out/r1e/mine_mixed.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
