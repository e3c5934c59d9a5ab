set -o pipefail
O=gpurun_out/r6ae
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
K=nodexa_chain_core_amd/kernels/equihash_ps.hsaco &&
cp $K $O/vop3.hsaco &&
for r in 1 2 3; do
  cp $O/vop3.hsaco $K &&
  timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 > $O/vop3_$r.json 2> $O/vop3_$r.err &&
  cp tools/bin/eqps_roundtrip.hsaco $K &&
  timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 > $O/plain_$r.json 2> $O/plain_$r.err || exit 1
done
cp $O/vop3.hsaco $K
echo "exit=$?"
