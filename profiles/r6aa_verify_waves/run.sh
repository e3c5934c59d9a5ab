set -o pipefail
O=gpurun_out/r6aa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_verify.py tests/test_gpu_resident_verify.py -v --timeout 200 --timeout-method thread > $O/pytest_verify.log 2>&1 &&
timeout -k 10 300 python3 -u tools/verify_light_timeline.py tests/data/testnet_mixed_10k.hdr 4 > $O/timeline.jsonl 2> $O/timeline.err
echo "exit=$?"
