"""Diagnostic: batch vs single-problem launches (bit-level)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "featuremetric-pnp_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import oracle.oracle as orc
from golden_io import case, maps64
from fmpnp import _lib, refine as rf

names = ["gm_c16", "behind_camera_gm", "odd_geom_gm", "no_support_init"]
probs = []
for nm in names:
    inp, meta, gold = case(nm)
    f, gx, gy = maps64(inp, orc.sobel)
    feats = rf.pack_features(torch.from_numpy(f), torch.from_numpy(gx), torch.from_numpy(gy), storage=torch.float64, device="cuda:0")
    probs.append(rf.make_problem(feats, torch.from_numpy(inp["fref"]), inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"], inp["R0"], inp["t0"]))

def run(ps, wgs=0, trace=True):
    opts = rf.make_options(20, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F64, wgs_per_problem=wgs)
    r, t = rf.refine(ps, opts, trace=trace)
    return r, t, _lib.last_launch()

rb, tb, lb = run(probs)
print("batch launch", lb)
rb2, tb2, _ = run(probs)
for i in range(4):
    print(i, "batch repeat equal:", np.array_equal(rb[i]["R"], rb2[i]["R"]))
for i, p in enumerate(probs):
    for w in (0, 1, 2, 8):
        r1, t1, l1 = run([p], wgs=w)
        d = np.abs(r1[0]["R"] - rb[i]["R"]).max()
        c1, cb = t1[0]["cost"], tb[i]["cost"]
        n = min(len(c1), len(cb))
        diff = np.nonzero(c1[:n] != cb[:n])[0]
        print(f"prob {i} wgs={w} launch={l1} maxdR={d:.3e} first cost diff at eval {diff[:3]} "
              f"({c1[diff[0]] if len(diff) else 0:.17g} vs {cb[diff[0]] if len(diff) else 0:.17g})")

print("--- batch variants ---")
r_single, t_single, _ = run([probs[0]], wgs=1)
for w in (1, 2, 8):
    r, t, l = run(probs, wgs=w)
    print(f"batch wgs={w} {l}: p0 equal single: {np.array_equal(r[0]['R'], r_single[0]['R'])}")
for reps in (2, 4, 8, 16):
    r, t, l = run([probs[0]] * reps, wgs=1)
    eq = [np.array_equal(x['R'], r_single[0]['R']) for x in r]
    print(f"{reps} copies wgs=1 {l}: equal single: {eq}")
    r, t, l = run([probs[0]] * reps, wgs=8)
    eq = [np.array_equal(x['R'], r_single[0]['R']) for x in r]
    print(f"{reps} copies wgs=8 {l}: equal single: {eq}")
