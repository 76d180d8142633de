#!/usr/bin/env python3
"""Summarise tools/gpu_profile_pyramid.sh: per pyramid level (the LM launches in dispatch order,
REPS per level; the first launch of each level excluded from the averages as a warm-up), the kernel,
the average duration (kernel trace) and the HBM bytes per launch (FETCH_SIZE doubled, gfx950;
WRITE_SIZE as is).  usage: pmc_pyramid_summary.py <dir> <N> <REPS>"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import ROOT, build_id  # noqa: E402

LEVELS = [(640, 1664), (128, 640), (0, 128)]


def lm_rows(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "lm_kernel" in r.get("Kernel_Name", "")]
    return rows


def main():
    d, N, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    tr = lm_rows(os.path.join(d, "trace", "**", "*kernel_trace.csv"))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = {}
    for name, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        rows = lm_rows(os.path.join(d, sub, "**", "*counter_collection.csv"))
        byd = {}
        for r in rows:
            if r["Counter_Name"] == name:
                k = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                byd[k] = byd.get(k, 0.0) + float(r["Counter_Value"])
        per[name] = [byd[k] for k in sorted(byd)]
    levels = []
    for li, (cb, ce) in enumerate(LEVELS):
        sl = slice(li * reps + 1, (li + 1) * reps)  # (launch 0 of the level: warm-up)
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr[sl]]
        f = per["FETCH_SIZE"][sl]
        w = per["WRITE_SIZE"][sl]
        b = (2 * sum(f) / len(f) + sum(w) / len(w)) * 1024
        ns = sum(durs) / len(durs)
        levels.append({"channels": [cb, ce], "kernel": tr[li * reps]["Kernel_Name"], "launches": len(durs),
                       "kernel_avg_ns": ns, "hbm_bytes_per_launch": int(b),
                       "achieved_GBps": round(b / ns, 1), "frac_of_8TBps": round(b / ns / 8000.0, 4)})
    out = {"workload": f"RobotCar pyramid, B=32, C=1664 256x256, N={N}, GM, 50 iters per level "
                       "(tools/pyramid_run.py)", "N": N, "levels": levels,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), KiB -> bytes",
           "source_digest": build_id().library_file_digest(os.environ.get("FMPNP_LIB_PATH")), "git_head": os.environ.get("GIT_HEAD") or None}
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
