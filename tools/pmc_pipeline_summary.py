#!/usr/bin/env python3
"""Summarise tools/gpu_profile_pipeline.sh: per fmpnp kernel family of the pipeline (f-only pack,
reference gather, LM), dispatches, average duration and HBM bytes (FETCH_SIZE doubled: gfx950
reports half of wide reads, MI355X_MICROARCH.md; WRITE_SIZE as is), and the totals per query.
usage: pmc_pipeline_summary.py <dir> <queries>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import ROOT, build_id  # noqa: E402


def family(name):
    if "hwc" in name or "pack" in name or "win_clear" in name or "win_mark" in name:
        return "pack"
    if "gather_ref" in name:
        return "gather_reference"
    if "lm_kernel" in name:
        return "lm"
    return None


def counter(d, sub, cname):
    tot = defaultdict(float)
    seen = defaultdict(set)
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            fam = family(r.get("Kernel_Name", ""))
            if fam and r.get("Counter_Name") == cname:
                tot[fam] += float(r["Counter_Value"])
                seen[fam].add(r.get("Dispatch_Id"))
    return tot, {k: len(v) for k, v in seen.items()}


def main():
    d, queries = sys.argv[1], int(sys.argv[2])
    stats = defaultdict(lambda: {"calls": 0, "total_ns": 0.0})
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            fam = family(r["Name"])
            if fam:
                stats[fam]["calls"] += int(r["Calls"])
                stats[fam]["total_ns"] += float(r["TotalDurationNs"])
    fetch, nf = counter(d, "pmc_fetch", "FETCH_SIZE")
    write, nw = counter(d, "pmc_write", "WRITE_SIZE")
    fams = {}
    for fam in ("pack", "gather_reference", "lm"):
        b = 2 * fetch.get(fam, 0.0) * 1024 + write.get(fam, 0.0) * 1024
        fams[fam] = {"dispatches": stats[fam]["calls"], "kernel_ns_per_query": stats[fam]["total_ns"] / queries,
                     "fetch_bytes_per_query": 2 * fetch.get(fam, 0.0) * 1024 / queries,
                     "write_bytes_per_query": write.get(fam, 0.0) * 1024 / queries,
                     "hbm_bytes_per_query": b / queries, "dispatches_counted": [nf.get(fam, 0), nw.get(fam, 0)]}
    robot = os.environ.get("ROBOTCAR") == "1"
    out = {"workload": "bench.py end_to_end robotcar_1664: RefinePipeline with 3 channel levels, 2 batches x 32 "
                       "queries of C = 1664 256x256 hypercolumns, N = 866 (tools/pipeline_run.py, ROBOTCAR=1)" if robot else
                       "bench.py end_to_end: RefinePipeline, 4 batches x 64 cfg2 queries from CHW hypercolumns "
                       "(f-only pack + reference gather + LM), tools/pipeline_run.py",
           "queries": queries, "window": int(os.environ.get("WINDOW", "0")) or None, "robotcar": robot,
           "families": fams,
           "hbm_bytes_per_query": sum(v["hbm_bytes_per_query"] for v in fams.values()),
           "kernel_ns_per_query": sum(v["kernel_ns_per_query"] for v in fams.values()),
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), KiB -> bytes",
           "source_digest": build_id().library_file_digest(os.environ.get("FMPNP_LIB_PATH")), "git_head": os.environ.get("GIT_HEAD") or None}
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
