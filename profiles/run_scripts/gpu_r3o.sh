#!/bin/bash
# r3o: Equihash PS: does a smaller batch (level footprint inside the Infinity Cache) pay per solve?
set -o pipefail
mkdir -p gpurun_out/r3o
cd "$GRAFT_REPO_ROOT" &&
for cfg in "2 ps" "4 ps" "2 ps:256" "4 ps:128" "8 ps" "16 ps:32"; do
  set -- $cfg
  timeout -k 10 120 python -u tools/equihash_bench.py --engines $2 --batches 6 --inst $1 >> gpurun_out/r3o/eb.log 2>&1 || exit 1
done
echo "exit=$?"
