set -o pipefail
O=gpurun_out/r6y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/valu_pmc -o vr --output-format csv -- tools/bin/valu_rates > $O/valu_rates.jsonl 2>&1
echo "exit=$?"
