#!/bin/bash
# hipGraph Equihash (kernels captured, clears as memsets): Equihash throughput graph vs direct, interleaved.
set -o pipefail
mkdir -p gpurun_out/r1u
for i in 1 2; do
  NODEXA_EQ_GRAPH=1 timeout -k 10 200 python -u tools/equihash_bench.py --inst 8 --batches 20 > gpurun_out/r1u/eq_graph_$i.log 2>&1 &&
  NODEXA_EQ_GRAPH=0 timeout -k 10 200 python -u tools/equihash_bench.py --inst 8 --batches 20 > gpurun_out/r1u/eq_direct_$i.log 2>&1 || exit $?
done
