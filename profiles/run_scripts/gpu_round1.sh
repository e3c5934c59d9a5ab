set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch;print(torch.cuda.get_device_name(0))" > gpurun_out/env.txt 2>&1
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench1.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
