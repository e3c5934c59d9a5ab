#!/bin/bash
# r4g: the Equihash mining loop with one solver+stream per slot (NODEXA_EQ_STREAMS=2) vs
# one shared (=1), with and without the one-rank RCCL group: per-step host timings and Sol/s
# (tools/eq_loop_probe.py); the Equihash GPU tests on the two-solver device.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_equihash_mining.py \
  > $O/pytest_eq.log 2>&1 || exit $?
for s in 1 2 1 2; do
  for c in "" --collectives; do
    NODEXA_EQ_STREAMS=$s timeout -k 10 200 python3 tools/eq_loop_probe.py $c \
      | sed "s/^{/{\"eq_streams\": $s, /" >> $O/eq_loop.jsonl 2>> $O/eq_loop.err || exit $?
  done
done
echo "exit=0"
