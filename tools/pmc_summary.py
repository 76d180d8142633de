#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run: per-kernel stats (kernel trace) and the HBM
bytes per LM launch from the FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB.  On gfx950 FETCH_SIZE
reports half of the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section):
it is doubled here; WRITE_SIZE is taken as is.

usage: pmc_summary.py <prof_dir> <batch> <out.json> [kernel name substring | auto] [tag]
(default "auto": the lm_kernel variant with the largest total time in the kernel trace --
the workload's LM launch, whichever specialisation the planner picked)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_id():
    """fmpnp/build_id.py loaded by path (no package import, no torch): the source digest bench.py
    checks a profile against."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "fmpnp_build_id", os.path.join(ROOT, "featuremetric-pnp_amd", "fmpnp", "build_id.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def rows(pattern):
    out = []
    for path in glob.glob(pattern, recursive=True):
        with open(path, newline="") as f:
            out.extend(csv.DictReader(f))
    return out


def counter_avg(prof, sub, name, kernel_key):
    vals = {}
    for r in rows(os.path.join(prof, sub, "**", "*counter_collection.csv")):
        if kernel_key in r.get("Kernel_Name", "") and r.get("Counter_Name") == name:
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    if not vals:
        return None, 0
    return sum(vals.values()) / len(vals), len(vals)


def main():
    prof, batch, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    key = sys.argv[4] if len(sys.argv) > 4 else "auto"
    tag = sys.argv[5] if len(sys.argv) > 5 else None
    stats = [r for r in rows(os.path.join(prof, "trace", "**", "*kernel_stats.csv"))]
    if key == "auto":
        lms = [r for r in stats if "lm_kernel" in r.get("Name", "")]
        lms.sort(key=lambda r: float(r.get("TotalDurationNs") or 0), reverse=True)
        key = lms[0]["Name"].replace("void ", "").split("(")[0] if lms else "lm_kernel"
    lm = [r for r in stats if key in r.get("Name", "")]
    fetch_kib, nf = counter_avg(prof, "pmc_fetch", "FETCH_SIZE", key)
    write_kib, nw = counter_avg(prof, "pmc_write", "WRITE_SIZE", key)
    summary = {
        "tag": tag,
        "batch": batch,
        "kernel": lm[0]["Name"] if lm else None,
        "kernel_calls": int(lm[0]["Calls"]) if lm else None,
        "kernel_avg_ns": float(lm[0]["AverageNs"]) if lm else None,
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib": write_kib,
        "dispatches_counted": [nf, nw],
        "hbm_bytes_per_launch": (None if fetch_kib is None or write_kib is None
                                 else int(2 * fetch_kib * 1024 + write_kib * 1024)),
        "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), KiB -> bytes",
        # the build the counters were taken with: bench.py uses the bytes only for this digest and
        # this kernel specialisation (GIT_HEAD: set by the caller; the box has no git history)
        "source_digest": build_id().library_file_digest(os.environ.get("FMPNP_LIB_PATH")),
        "git_head": os.environ.get("GIT_HEAD") or None,
        "all_kernels": [{k: r[k] for k in ("Name", "Calls", "AverageNs", "Percentage") if k in r} for r in stats],
    }
    with open(out, "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "all_kernels"}))


if __name__ == "__main__":
    main()
