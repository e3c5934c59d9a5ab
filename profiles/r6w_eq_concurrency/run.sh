set -o pipefail
O=gpurun_out/r6w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u tools/eq_concurrency.py --configs 16:16:1 16:16:2 16:16:3 32:8:1 --solves 1024 --reps 3 > $O/eq_conc.jsonl 2> $O/eq_conc.err
echo "exit=$?"
