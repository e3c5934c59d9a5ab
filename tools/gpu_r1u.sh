#!/bin/bash
# hipGraph Equihash: agreement test, then graph vs direct launches in the bench.
set -o pipefail
mkdir -p gpurun_out/r1u
timeout -k 10 300 python -u -m pytest tests/test_gpu_equihash.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r1u/pytest_eq.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r1u/bench_graph.log 2>&1 &&
NODEXA_EQ_GRAPH=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r1u/bench_direct.log 2>&1
