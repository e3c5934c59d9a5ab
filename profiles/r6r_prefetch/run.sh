set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_verify.py tests/test_gpu_resident_verify.py -v --timeout 200 --timeout-method thread > $O/pytest_verify.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo "exit=$?"
