#!/bin/bash
# r4b: (1) the new GPU tests — device-resident batch header verify, Equihash mined by the node,
# device-side solution verdicts, the
# one-rank RCCL world (DAG gather, mining loop + injected abort, batch verify) — and the miner
# tests that moved to the one mining loop; (2) the pointer-path (epoch 390, DAG > 4 GiB) digest
# variants, to retire the LDS-digest form; (3) bench.py plain and with one-rank RCCL collectives,
# and a kernel trace of the RCCL run (RCCL kernels interleaved with kawpow_search).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_resident_verify.py tests/test_gpu_equihash_mining.py tests/test_gpu_rccl.py \
  tests/test_gpu_node_miner.py tests/test_gpu_kawpow.py tests/test_gpu_multirank.py > $O/pytest_new.log 2>&1
rc=$?; echo "pytest=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
P390="KP_HASHES=1,KP_DPP,KP_BARRETT,KP_L1X4,KP_BLOCK=512,KP_NT_DAG,KP_SCHED_FENCE"
timeout -k 10 400 python3 -u tools/kawpow_sweep.py --epoch 390 --batch 8388608 --rounds 5 --raw \
  --variants "$P390" "$P390,KP_DIGEST_REG" "${P390/KP_BLOCK=512/KP_BLOCK=768},KP_DIGEST_REG,KP_MIN_WAVES=6" \
  --out $O/sweep390.json > $O/sweep390.log 2>&1
rc=$?; echo "sweep=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --collectives > $O/bench_rccl.json 2> $O/bench_rccl.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o rccl \
  -- python3 bench.py --steps 6 --warmup 2 --collectives --verify 0 > $O/prof_rccl.log 2>&1
echo "bench=$?"
