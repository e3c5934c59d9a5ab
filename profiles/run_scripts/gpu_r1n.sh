#!/bin/bash
# Dense DAG-mode batch verify: GPU numerics tests + verify bench on the mixed fixture.
set -o pipefail
mkdir -p gpurun_out/r1n
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r1n/pytest_verify.log 2>&1 &&
timeout -k 10 300 python -u tools/verify_bench.py --cpu-sample 10 > gpurun_out/r1n/verify_bench.log 2>&1
