set -e
mkdir -p gpurun_out/r6b
V1="KP_HASHES=1,KP_DPP,KP_BARRETT,KP_L1X4,KP_BLOCK=512,KP_NT_DAG,KP_SCHED_FENCE"
V2="KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE,KP_SBUFFER_HI"
V3="KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=512,KP_NT_DAG,KP_SCHED_FENCE,KP_SBUFFER_HI"
timeout -k 10 300 python tools/kawpow_sweep.py --epoch 390 --raw --rounds 9 --batch 33554432 --variants "$V1" "$V2" "$V3" --out gpurun_out/r6b/e390.json > gpurun_out/r6b/e390.log 2>&1
timeout -k 10 300 python tools/kawpow_sweep.py --epoch 384 --rounds 9 --batch 33554432 --variants tuned --out gpurun_out/r6b/e384.json > gpurun_out/r6b/e384.log 2>&1
