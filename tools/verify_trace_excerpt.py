"""One resident-verify run out of a rocprofv3 kernel + memory-copy trace (tools/gpu_r4z11.sh): the
kernels and copies of the second-to-last run (from its upload to the next run's upload), times
in us relative to the upload's start. Usage: verify_trace_excerpt.py <trace dir> > excerpt.csv"""
import csv
import glob
import os
import sys


def rows(d, suffix):
    path = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    return list(csv.DictReader(open(path[0]))) if path else []


def main(d: str) -> None:
    ev = []
    for r in rows(d, "kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel", r["Kernel_Name"].split("(")[0],
                   r.get("Queue_Id", ""), ""))
    for r in rows(d, "memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy",
                   r.get("Direction", "").replace("MEMORY_COPY_", ""), "", r.get("Stream_Id", "")))
    ev.sort()
    # a run: from the upload before its kawpow_mixonly_batch to the upload of the next run
    mo = [i for i, e in enumerate(ev) if e[3] == "kawpow_mixonly_batch"]
    if len(mo) < 3:
        sys.exit("fewer than three runs in the trace")

    def upload_before(i):
        while i > 0 and not (ev[i][2] == "copy" and ev[i][3] == "HOST_TO_DEVICE"):
            i -= 1
        return i

    i0, i1 = upload_before(mo[-2]), upload_before(mo[-1])
    t0 = ev[i0][0]
    out = csv.writer(sys.stdout)
    out.writerow(["start_us", "end_us", "kind", "name", "queue", "stream"])
    for e in ev[i0:i1]:
        out.writerow([round((e[0] - t0) / 1e3, 1), round((e[1] - t0) / 1e3, 1), e[2], e[3], e[4], e[5]])


if __name__ == "__main__":
    main(sys.argv[1])
