set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/pmc_tcc -o pmc --output-format csv -- tools/bin/dag_build_probe > $O/pmc_tcc.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- tools/bin/dag_build_probe > $O/pmc_sq.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/bench_prof -o bench --output-format csv -- python3 -u bench.py --steps 5 --warmup 1 > $O/bench_prof.json 2> $O/bench_prof.err
echo "exit=$?"
