set -o pipefail
O=gpurun_out/r6ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/light_tcc -o lt --output-format csv -- python3 -u tools/verify_light_timeline.py tests/data/testnet_mixed_10k.hdr 2 > $O/light_tcc.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/light_sq -o lt --output-format csv -- python3 -u tools/verify_light_timeline.py tests/data/testnet_mixed_10k.hdr 2 > $O/light_sq.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/bench_prof -o bench --output-format csv -- python3 -u bench.py > $O/bench_prof.json 2> $O/bench_prof.err
echo "exit=$?"
