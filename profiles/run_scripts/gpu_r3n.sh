#!/bin/bash
# r3n: Equihash PS bound analysis: no row stores / no back-pointer copies / dense emission.
set -o pipefail
mkdir -p gpurun_out/r3n
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python -u tools/equihash_bench.py --engines ps --batches 6 --variants "" EQP_DENSE EQP_NO_STORE EQP_NO_REFS EQP_NO_STORE,EQP_NO_REFS > gpurun_out/r3n/eb.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n/prof_ns -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 4 --variants EQP_NO_STORE > gpurun_out/r3n/prof_ns.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n/prof_base -o eq --output-format csv -- python3 tools/equihash_bench.py --engines ps --batches 4 > gpurun_out/r3n/prof_base.log 2>&1
echo "exit=$?"
