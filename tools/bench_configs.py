"""Per-config measurements beside the headline bench (BASELINE.json configs[0..4]).

Each line: config, batch, ms per launch, pose-refinements/s, GN-iters/s.  Synthetic inputs
(SURVEY.md 8d recipe).  configs[3] (the pyramid) runs its three levels as three launches
(coarse to fine, the pose chained: model.py:178-213 with one map per level).

python tools/bench_configs.py [--quick]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd")]
import torch  # noqa: E402

from fmpnp import _lib, refine as rf, synth  # noqa: E402

DEV = torch.device("cuda", 0)


def build(N, C, H, W, B, seed0=0):
    probs = []
    for q in range(B):
        inp = synth.problem_inputs(N, C, H, W, seed=seed0 + q, device=DEV)
        feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=DEV)
        probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                     inp["R0"], inp["t0"]))
        del inp
    return probs


def time_batch(probs, opts, reps=5):
    ab = rf.AsyncBatch(probs, opts)
    ab.launch()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        ab.launch()
    e.record()
    torch.cuda.synchronize()
    res = ab.results()
    return s.elapsed_time(e) / reps, _lib.last_launch(), sorted({r["status"] for r in res})


def report(name, B, iters, ms, launch, statuses, extra=None):
    d = dict(config=name, batch=B, iters=iters, ms_per_launch=round(ms, 4),
             pose_refinements_per_s=round(B / (ms / 1e3), 1), gn_iters_per_s=round(B * iters / (ms / 1e3), 1),
             launch=launch, statuses=statuses)
    d.update(extra or {})
    print(json.dumps(d), flush=True)


def main():
    quick = "--quick" in sys.argv
    # configs[0]: toy shape (N=64, C=3, 120x160, squared, 20 iters)
    for B in (1, 128):
        probs = build(64, 3, 120, 160, B)
        ms, la, st = time_batch(probs, rf.make_options(20, 0.01, _lib.SQUARED, dtype=_lib.F32))
        report("configs[0] toy shape", B, 20, ms, la, st)
    # configs[1]: one query, N=512, C=256, 240x320, GM, 50 iters
    probs = build(512, 256, 240, 320, 1)
    ms, la, st = time_batch(probs, rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32))
    report("configs[1] single query", 1, 50, ms, la, st)
    del probs
    # configs[3]: 3-level pyramid, one map per level, coarse to fine, pose chained
    B = 8 if quick else 32
    levels = [(512, 120, 160), (256, 240, 320), (128, 480, 640)]
    per_level = []
    t_total = 0.0
    for (C, H, W) in levels:
        probs = []
        for q in range(B):
            # same scene (points, K scaled to the 4x-stride image of this level is not used: the
            # image is fixed at 2560x1920) -> points from the finest level's scene
            inp = synth.problem_inputs(512, C, H, W, seed=q, device=DEV)
            feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=DEV)
            probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"],
                                         inp["im_height"], inp["R0"], inp["t0"]))
            del inp
        ms, la, st = time_batch(probs, rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32))
        per_level.append(dict(C=C, H=H, W=W, ms=round(ms, 4), launch=la))
        t_total += ms
        del probs
        torch.cuda.empty_cache()
    report("configs[3] 3-level pyramid (sum of the three level launches)", B, 150, t_total, None, [],
           {"levels": per_level})
    # configs[4]: N=2048, C=512, 480x640, Cauchy, 50 iters (1.9 GB packed map per query)
    for B in ((1, 8) if quick else (1, 32)):
        probs = build(2048, 512, 480, 640, B)
        ms, la, st = time_batch(probs, rf.make_options(50, 0.01, _lib.CAUCHY, dtype=_lib.F32), reps=3)
        report("configs[4] 2048 pts C=512 480x640 Cauchy", B, 50, ms, la, st)
        del probs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(json.dumps({"wall_s": round(time.time() - t0, 1)}))
