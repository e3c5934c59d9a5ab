#!/bin/bash
# r5b: the coarse-bucket Equihash engine (equihash_cb.hip): exactness against the golden solver,
# interleaved timing against the private-slot engine at the mining window's 16 instances, kernel
# stats and EA requests per kernel; kawpow_verify_waves with its program words in SGPRs: the
# bit-exactness test against the LDS interpreter and the verify pipeline's kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_equihash.py -v --timeout 120 --timeout-method thread \
  > $O/pytest_eq.log 2>&1
rc=$?; [ $rc -le 1 ] || { echo "pytest rc=$rc: stop"; exit $rc; }  # test failures go on; faults / timeouts stop
timeout -k 10 300 python3 -u tools/equihash_bench.py --inst 16 --batches 8 --engines cb ps > $O/eq16.jsonl 2> $O/eq16.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o eq --output-format csv \
  -- python3 tools/equihash_bench.py --inst 16 --batches 4 --engines cb > $O/prof.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum -d $O/pmc -o eq \
  --output-format csv -- python3 tools/equihash_bench.py --inst 16 --batches 1 --engines cb > $O/pmc.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_resident_verify.py -v -x --timeout 120 --timeout-method thread \
  > $O/pytest_verify.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_verify -o v --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --equihash 0 --verify 1 > $O/prof_verify.log 2>&1
echo "exit=$?"
