"""Timeline of the streamed pipeline's last pass (tools/pipeline_run.py under rocprofv3 --kernel-trace, the
SQLite output): the pass's span, each kernel family's busy time, the idle gaps of the GPU and the LM
launches' overlap with the preparation kernels.

  python tools/pipe_timeline_db.py gpurun_out/pipe_tl/run_results.db [n_lm_launches_per_pass=4]
"""
import sqlite3
import sys


def family(name):
    for key, fam in (("lm_kernel", "lm"), ("hwc_win", "pack_win"), ("hwc", "pack"), ("sobel_pack", "pack"),
                     ("gather_ref", "gather"), ("win_mark", "mark"), ("win_clear", "clear")):
        if key in name:
            return fam
    return "other"


def union(iv):
    tot, cur = 0, None
    for a, b in sorted(iv):
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def main():
    db, per = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4
    c = sqlite3.connect(db)
    k = sorted((s, e, n) for n, s, e in c.execute("select name, start, end from kernels"))
    lm = [x for x in k if "lm_kernel" in x[2]]
    t_end = lm[-1][1]
    prev_end = lm[-per - 1][1] if len(lm) > per else k[0][0]
    win = [x for x in k if x[0] >= prev_end and x[1] <= t_end and family(x[2]) != "other"]
    t0 = min(x[0] for x in win)
    span = t_end - t0
    print(f"last pass: {len(win)} kernels, span {span / 1e6:.3f} ms")
    fams = {}
    for s, e, n in win:
        fams.setdefault(family(n), []).append((s, e))
    for f, iv in sorted(fams.items()):
        print(f"  {f:9s} n {len(iv):4d}  busy {union(iv) / 1e6:7.3f} ms  sum {sum(e - s for s, e in iv) / 1e6:7.3f} ms")
    prep = [iv for f, v in fams.items() if f != "lm" for iv in v]
    allk = [(s, e) for s, e, _ in win]
    print(f"  GPU busy (any kernel) {union(allk) / 1e6:.3f} ms, idle {(span - union(allk)) / 1e6:.3f} ms; "
          f"preparation busy {union(prep) / 1e6:.3f} ms")
    # first preparation kernel -> first LM launch (the fill), last prep kernel -> end (the drain)
    lms = sorted(fams.get("lm", []))
    print(f"  fill (first kernel -> first LM start) {(lms[0][0] - t0) / 1e6:.3f} ms; drain (last prep end -> "
          f"end) {(t_end - max(e for s, e in prep)) / 1e6:.3f} ms")
    for i, (s, e) in enumerate(lms):
        print(f"  LM {i}: start {(s - t0) / 1e6:7.3f} end {(e - t0) / 1e6:7.3f} ({(e - s) / 1e6:.3f} ms)")


if __name__ == "__main__":
    main()
