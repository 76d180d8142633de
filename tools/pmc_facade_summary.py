#!/usr/bin/env python3
"""Summarise tools/gpu_profile_facade.sh: the reference consumer's per-call path (fmpnp.feature_pnp one
query per call, tools/facade_call.py) per kernel family -- pack, reference gather, compute_cost, LM,
window marking, runtime copies -- dispatches per call, kernel ns per call and HBM bytes per call
(FETCH_SIZE x2, MI355X_MICROARCH.md; WRITE_SIZE as is), with the wall-clock ms per call of the trace run.
usage: pmc_facade_summary.py <dir> <shape> <calls in the trace run> <calls in each counter run>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import build_id  # noqa: E402

FAMS = ("pack", "gather_reference", "compute_cost", "lm", "window", "runtime")


def family(name):
    if "sobel_pack" in name or "hwc" in name:
        return "pack"
    if "gather_ref" in name:
        return "gather_reference"
    if "point_cost" in name or "cost_mean" in name:
        return "compute_cost"
    if "lm_kernel" in name:
        return "lm"
    if "win_clear" in name or "win_mark" in name:
        return "window"
    if "rocclr" in name:
        return "runtime"
    return None


def counter(d, sub, cname):
    tot = defaultdict(float)
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            fam = family(r.get("Kernel_Name", ""))
            if fam and r.get("Counter_Name") == cname:
                tot[fam] += float(r["Counter_Value"])
    return tot


def main():
    d, shape, n_trace, n_pmc = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    stats = defaultdict(lambda: {"calls": 0, "total_ns": 0.0})
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            fam = family(r["Name"])
            if fam:
                stats[fam]["calls"] += int(r["Calls"])
                stats[fam]["total_ns"] += float(r["TotalDurationNs"])
    fetch = counter(d, "pmc_fetch", "FETCH_SIZE")
    write = counter(d, "pmc_write", "WRITE_SIZE")
    wall = None
    try:
        with open(os.path.join(d, "trace.json")) as f:
            wall = json.loads(f.read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        pass
    fams = {}
    for fam in FAMS:
        if fam not in stats:
            continue
        fams[fam] = {"dispatches_per_call": stats[fam]["calls"] / n_trace,
                     "kernel_us_per_call": round(stats[fam]["total_ns"] / n_trace / 1e3, 2),
                     "fetch_bytes_per_call": round(2 * fetch.get(fam, 0.0) * 1024 / n_pmc),
                     "write_bytes_per_call": round(write.get(fam, 0.0) * 1024 / n_pmc)}
        fams[fam]["hbm_bytes_per_call"] = fams[fam]["fetch_bytes_per_call"] + fams[fam]["write_bytes_per_call"]
    kern_us = sum(v["kernel_us_per_call"] for v in fams.values())
    out = {"workload": f"fmpnp.feature_pnp, one query per call, {shape} (tools/facade_call.py; "
                       "sparse_to_dense_predictor.py:242-247 times one optimize_feature_pnp call per query)",
           "shape": shape, "families": fams, "kernel_us_per_call": round(kern_us, 2),
           "hbm_bytes_per_call": sum(v["hbm_bytes_per_call"] for v in fams.values()),
           "wall_ms_per_call_trace_run": wall.get("ms_per_call") if wall else None,
           "wall_over_kernels": round(wall["ms_per_call"] * 1e3 / kern_us, 3) if wall and kern_us else None,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving; scattered reads: profiles/r05_scatter_fetch_"
                         "calibration.txt), KiB -> bytes; the counter runs' calls include their warm-up calls",
           "source_digest": build_id().library_file_digest(os.environ.get("FMPNP_LIB_PATH"))}
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
