set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python3 -u tools/verify_light_timeline.py tests/data/testnet_mixed_10k.hdr 5 > $O/timeline.jsonl 2> $O/timeline.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o lt --output-format csv -- python3 -u tools/verify_light_timeline.py tests/data/testnet_mixed_10k.hdr 3 > $O/timeline_prof.jsonl 2> $O/timeline_prof.err
echo "exit=$?"
