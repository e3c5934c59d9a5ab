#!/bin/bash
# r5 final: the whole GPU tier, smoke(), the driver-contract bench, kernel stats, X16R probes after the verify stream changes
# bench (with GPU clock/power provenance and the device-clock rate), kernel stats of a short bench
# and of the verify pipeline.
set -o pipefail
O=gpurun_out/r5final
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv \
  -- python3 bench.py --steps 6 --warmup 2 > $O/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_verify -o v --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --equihash 0 --verify 1 > $O/prof_verify.log 2>&1 &&
timeout -k 10 300 python3 -u tools/x16r_probe.py --n 65536 --reps 3 > $O/x16r_probe.json 2> $O/x16r_probe.err &&
  timeout -k 10 200 python3 -u tools/x16r_slot_probe.py --n 65536 > $O/x16r_slots65k.json 2> $O/x16r_slots.err
echo "exit=$?"
