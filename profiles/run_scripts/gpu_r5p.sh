#!/bin/bash
# r5p: the jump-table dispatch on its own (tools/jump_table_probe.py, prebuilt tools/jt.hsaco)
set -o pipefail
O=gpurun_out/r5p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 5 90 python3 -u tools/jump_table_probe.py > $O/jt.json 2> $O/jt.err
echo "exit=$?"
