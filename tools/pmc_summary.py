#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel dispatch into JSON.

    python tools/pmc_summary.py gpurun_out/pmc2/sq_counter_collection.csv [more.csv] > out.json

For kawpow_search dispatches it also derives per-hash figures (one hash per
grid thread): VALU / LDS wave-instructions per hash, effective DAG bandwidth
(16 KiB of gathers per hash) and a VALU-issue utilisation estimate assuming 4
cycles per wave64 integer VALU instruction on the 1024 SIMDs at 2.4 GHz.
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict


def load(paths: list[str]) -> list[dict]:
    rows: dict[tuple, dict] = defaultdict(dict)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                key = (p.rsplit("/", 1)[-1].split("_")[0], int(r["Dispatch_Id"]))
                d = rows[key]
                d.update(kernel=r["Kernel_Name"], dispatch=int(r["Dispatch_Id"]), grid=int(r["Grid_Size"]),
                         workgroup=int(r["Workgroup_Size"]), vgpr=int(r["VGPR_Count"]), lds=int(r["LDS_Block_Size"]),
                         dur_ms=(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = []
    for d in rows.values():
        if d["kernel"] == "kawpow_search" and d["grid"] >= 1 << 20:
            hashes = d["grid"]
            if "SQ_INSTS_VALU" in d:
                d["valu_wave_instr_per_hash"] = round(d["SQ_INSTS_VALU"] / hashes, 1)
                d["valu_issue_util_4cyc"] = round(d["SQ_INSTS_VALU"] * 4 / (1024 * 2.4e9 * d["dur_ms"] / 1e3), 3)
            if "SQ_INSTS_LDS" in d:
                d["lds_wave_instr_per_hash"] = round(d["SQ_INSTS_LDS"] / hashes, 1)
            d["mhs"] = round(hashes / (d["dur_ms"] / 1e3) / 1e6, 1)
            d["dag_TBps_effective"] = round(hashes * 16384 / (d["dur_ms"] / 1e3) / 1e12, 2)
        out.append(d)
    out.sort(key=lambda d: (d["kernel"], d["dispatch"]))
    return out


if __name__ == "__main__":
    json.dump(load(sys.argv[1:]), sys.stdout, indent=1)
    print()
