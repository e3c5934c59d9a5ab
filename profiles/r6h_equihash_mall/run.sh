mkdir -p gpurun_out/r6h
timeout -k 10 300 python bench.py > gpurun_out/r6h/bench1.json 2> gpurun_out/r6h/bench1.err && \
for n in 16 8 4 2 1; do timeout -k 10 120 python tools/equihash_bench.py --inst $n --batches 6 >> gpurun_out/r6h/eq_inst.jsonl 2>> gpurun_out/r6h/eq.err || exit 1; done
