mkdir -p gpurun_out/r6i
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > gpurun_out/r6i/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r6i/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6i/smoke.log 2>&1 && \
NODEXA_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 > gpurun_out/r6i/bench2.json 2> gpurun_out/r6i/bench2.err
