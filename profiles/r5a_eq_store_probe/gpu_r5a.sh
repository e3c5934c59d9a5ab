#!/bin/bash
# r5a: Equihash coarse-bucket / run-buffer memory-pattern probe (tools/eq_runs_probe.hip): write
# rates and EA requests per row for D destinations x RR-row LDS run buffers, and K-fold re-reads of
# coarse buckets; then the resident-verify GPU tests (ADVICE r4 fixes) and a baseline bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 120 tools/bin/eq_runs_probe > $O/probe.jsonl 2> $O/probe.err &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum -d $O/pmc -o p \
  --output-format csv -- tools/bin/eq_runs_probe > $O/pmc.log 2>&1 &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_verify.py -v --timeout 120 --timeout-method thread \
  > $O/pytest_resident.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo "exit=$?"
