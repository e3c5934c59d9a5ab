#!/bin/bash
# r4f: one stream per search slot (the queued window fills the running window's tail) against both
# slots on one stream, interleaved bench runs (KawPow only), plus the GPU tests of the loop.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_kawpow.py::test_pipelined_search_loop_on_gpu tests/test_gpu_node_miner.py tests/test_gpu_rccl.py \
  > $O/pytest.log 2>&1 || exit $?
for v in 1 2 1 2 1 2; do
  NODEXA_SEARCH_STREAMS=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 4 --equihash 0 --verify 0 \
    > $O/bench_s$v.$(date +%s).json 2>> $O/bench_s$v.err || exit $?
done
# kernel time of the resident verify pipeline (BASELINE config 5)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_verify -o v \
  -- python3 bench.py --steps 2 --warmup 1 --equihash 0 --verify 1 > $O/prof_verify.log 2>&1 || exit $?
echo "exit=0"
