set -o pipefail
O=gpurun_out/r6ai
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 900 python3 -u tools/equihash_bench.py --inst 16 --batches 8 --engines ps --variants "" " -mllvm:-amdgpu-use-amdgpu-trackers" " -mllvm:-amdgpu-sched-strategy=max-ilp" " -mllvm:-amdgpu-schedule-metric-bias=0" " -mllvm:-misched-postra" > $O/eqb.log 2>&1
echo "exit=$?"
