mkdir -p gpurun_out/r6l
T="KP_HASHES=1,KP_DPP,KP_BARRETT,KP_SBUFFER,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE"
P="KP_HASHES=1,KP_DPP,KP_BARRETT,KP_PTR64,KP_L1X4,KP_BLOCK=768,KP_MIN_WAVES=6,KP_NT_DAG,KP_SCHED_FENCE"
timeout -k 10 60 tools/bin/valu_rates > gpurun_out/r6l/valu_rates.jsonl 2>&1 && \
timeout -k 10 400 python tools/kawpow_sweep.py --epoch 384 --raw --rounds 11 --batch 33554432 --variants "$T" "$T,KP_PARK_SEED" "$T,KP_KISS_ASM" "$T,KP_PARK_SEED,KP_KISS_ASM" --out gpurun_out/r6l/e384.json > gpurun_out/r6l/e384.log 2>&1 && \
timeout -k 10 400 python tools/kawpow_sweep.py --epoch 390 --raw --rounds 11 --batch 33554432 --variants "$P" "$P,KP_PARK_SEED,KP_KISS_ASM" --out gpurun_out/r6l/e390.json > gpurun_out/r6l/e390.log 2>&1
