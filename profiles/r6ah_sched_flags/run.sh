set -o pipefail
O=gpurun_out/r6ah
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 1000 python3 -u tools/kawpow_sweep.py --raw --epoch 384 --rounds 7 --batch 33554432 --check-windows 2 --variants "KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE" "KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE,-mllvm:-amdgpu-use-amdgpu-trackers" "KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE,-mllvm:-amdgpu-schedule-metric-bias=100" "KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE,-mllvm:-amdgpu-schedule-metric-bias=0" "KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE,-mllvm:-misched-postra" "KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE,-mllvm:-amdgpu-sched-strategy=iterative-ilp" --out $O/sweep.json > $O/sweep.log 2>&1
echo "exit=$?"
