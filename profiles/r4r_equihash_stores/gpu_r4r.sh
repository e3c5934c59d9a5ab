#!/bin/bash
# r4r: where the Equihash rounds' EA write requests come from: the base build against one with the
# row stores compiled out (EQP_NO_ROW_STORE, results not collected), EA write requests and bytes
# per kernel, and the kernel times of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4r
mkdir -p $O
for v in base EQP_NO_ROW_STORE; do
  arg=""; [ "$v" != base ] && arg="--variant $v"
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/req_$v -o eq \
    --output-format csv -- python3 tools/eq_store_probe.py $arg > $O/req_$v.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/size_$v -o eq \
    --output-format csv -- python3 tools/eq_store_probe.py $arg > $O/size_$v.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/time_$v -o eq \
    --output-format csv -- python3 tools/eq_store_probe.py $arg --launches 4 > $O/time_$v.log 2>&1 || exit $?
done
echo "exit=0"
