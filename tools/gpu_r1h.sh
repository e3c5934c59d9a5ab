#!/bin/bash
# Mixed KawPow+Equihash synthetic chain (BASELINE config 5), its batch-verify bench, and an
# Equihash instances-per-batch sweep (MALL residency vs parallelism).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1h gpurun_out/data
for n in 2 4 8 16; do
  timeout -k 10 120 python -u tools/equihash_bench.py --inst $n --batches 6 > gpurun_out/r1h/eq_inst$n.log 2>&1 || exit $?
done
timeout -k 10 700 python -u tools/make_synthetic_chain.py --n 9000 --equihash 1000 --backend gpu --out gpurun_out/data/testnet_mixed_10k.hdr > gpurun_out/r1h/mine_mixed.log 2>&1 && \
timeout -k 10 200 python -u tools/verify_bench.py --file gpurun_out/data/testnet_mixed_10k.hdr --cpu-sample 10 > gpurun_out/r1h/verify_bench_mixed.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
