set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python3 -u tools/kawpow_sweep.py --epoch 384 --rounds 3 --batch 8388608 --check-windows 1 --out $O/sweep.json > $O/sweep.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $O/kp_pmc -o kp --output-format csv -- python3 tools/kawpow_sweep.py --epoch 384 --rounds 2 --batch 8388608 --check-windows 1 > $O/kp_pmc.log 2>&1
echo "exit=$?"
