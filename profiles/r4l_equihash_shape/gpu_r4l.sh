#!/bin/bash
# r4l: Equihash with writers per instance sized to fill the CUs (16 at the mining window's 16
# instances) and a 256-wide final round: the exactness and mining GPU tests, then the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_equihash.py \
  tests/test_gpu_equihash_mining.py tests/test_gpu_eq_graph.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
# producer threads per round workgroup (EQP_NP) re-swept in the new shape (r4m)
timeout -k 10 500 python3 tools/equihash_bench.py --inst 16 --batches 10 --engines ps:16:1024:256 \
  --variants "" EQP_NP=384 EQP_NP=512 EQP_NP=576 > $O/eq_np.jsonl 2> $O/eq_np.err || exit $?
# EA write requests per kernel in the 16-writer shape (r4c: the 32-writer shape at 8 instances)
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/pmc16 -o eq \
  --output-format csv -- python3 tools/equihash_bench.py --engines ps --inst 16 --batches 1 > $O/pmc16.log 2>&1 || exit $?
echo "exit=0"
