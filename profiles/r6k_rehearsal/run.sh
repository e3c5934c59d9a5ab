set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 60 tools/bin/valu_rates > $O/valu_rates.jsonl 2>&1 &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv \
  -- python3 bench.py --steps 6 --warmup 2 > $O/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_verify -o v --output-format csv \
  -- python3 bench.py --steps 2 --warmup 1 --equihash 0 --verify 1 > $O/prof_verify.log 2>&1
echo "exit=$?"
