set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 600 python3 -u tools/kawpow_sweep.py --epoch 384 --rounds 9 --batch 33554432 --check-windows 4 --objects roundtrip=tools/bin/kp_p960041_roundtrip.hsaco e64=tools/bin/kp_p960041_e64.hsaco --out $O/sweep.json > $O/sweep.log 2>&1
echo "exit=$?"
