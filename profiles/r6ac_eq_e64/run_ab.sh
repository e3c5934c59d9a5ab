set -o pipefail
O=gpurun_out/r6ac
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python3 -u - > $O/eq_e64.jsonl 2> $O/eq_e64.err <<'PY'
import json, os, statistics, sys, time
sys.path.insert(0, os.getcwd())
import torch
from nodexa_chain_core_amd.ops.equihash import EquihashSolver
BIN = "tools/bin"
objs = {"engine": None, "roundtrip": os.path.join(BIN, "eqps_roundtrip.hsaco"), "e64": os.path.join(BIN, "eqps_e64.hsaco")}
solvers = {k: EquihashSolver(num_inst=16, device=0, code_object=v) for k, v in objs.items()}
base = bytes(range(108))
mk = lambda t, i, j: base + bytes([t, i & 255, (i >> 8) & 255, j])
windows = 24
times = {k: [] for k in objs}
sols = {k: 0 for k in objs}
for rnd in range(6):
    items = list(solvers.items())
    items = items[rnd % 3:] + items[:rnd % 3]
    for k, sv in items:
        t = list(objs).index(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(windows):
            sv.launch([mk(t, rnd * windows + i, j) for j in range(16)])
            if i >= 1:
                sols[k] += sum(len(x) for x in sv.collect_arrays(verify="device"))
        sols[k] += sum(len(x) for x in sv.collect_arrays(verify="device"))
        torch.cuda.synchronize()
        times[k].append((time.perf_counter() - t0) / (windows * 16) * 1e3)
for k in objs:
    print(json.dumps({"object": k, "ms_per_solve_median": round(statistics.median(times[k][1:]), 4),
                      "ms_per_solve": [round(x, 4) for x in times[k]], "solutions": sols[k],
                      "fallbacks": solvers[k].fallbacks}), flush=True)
PY
echo "exit=$?"
