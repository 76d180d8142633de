"""Every LM kernel specialisation the launch planner can choose, checked against the oracle.

Per launch the planner (featuremetric-pnp_amd/csrc/fmpnp_api.hip make_plan) picks one compiled
specialisation of the LM kernel -- (texel dtype, build, team, ratio, variant), reported by
fmpnp_plan / fmpnp_last_launch_info:

  build    latency (512-thread workgroups), throughput (two 256-thread workgroups per CU, batches
           of >= 2 problems per CU), wide (one wave per SIMD: the bilinear cell memo);
  team     several workgroups per problem (cross-workgroup exchange compiled in);
  ratio    the ratio test (featurePnP/model.py:120-129,324-336);
  variant  loss / sampling / layout specialisation, speculative gathers (_SPEC) and the
           first-evaluation helpers' hand-off (_H).

This file
  1. sweeps the planner over a grid of batch sizes, problem sizes and options (fmpnp_plan: no
     launch) and collects every specialisation it chooses;
  2. runs, for every specialisation in CASES, a 50-iteration refinement of small synthetic
     problems that the planner sends to exactly that specialisation (asserted through
     fmpnp_last_launch_info) and compares it with the oracle (oracle/fmpnp_oracle.c, the C
     restatement of featurePnP/model.py:245-494) on the same inputs;
  3. asserts that every specialisation of the sweep has a case in CASES, and every case is one
     the planner chooses.

Tolerances: fp64 texels -- identical per-evaluation support counts and evaluation count, costs
within 1e-10 relative, poses within 1e-9 (the golden-vector tolerances); fp32 texels -- identical
support counts and evaluation count, costs within 1e-6 relative, final pose within 1e-4 rad /
1e-4 m (BASELINE.json north star).
"""
import itertools
import math

import numpy as np
import pytest
import torch

import oracle.oracle as orc

pytestmark = pytest.mark.gpu

from fmpnp import _lib, refine as rf, synth  # noqa: E402  (no skip: a missing HIP library must fail)

DEV = "cuda:0"
ITERS = 50
N_PTS, C, HF, WF = 128, 16, 48, 64        # small problems: two 64-point blocks, 4x image
N_512 = 480                               # the _512 recipes: 449..512 points (eight blocks, the last partial)
M512 = ("gm_spec_512", "gm_spec_h_512")
LOSSES = {"gm": (_lib.GEMAN_MCCLURE, "geman_mcclure"), "cauchy": (_lib.CAUCHY, "cauchy")}

# recipe name -> (B, loss, mode, sampling, layout, memo, speculate, wgs_per_problem, variant,
#                 build, team).  Each recipe runs with ratio off / 0.8 and fp32 / fp64 texels
#                 (layout "f" is fp32 only).
RECIPES = {
    # latency build, one workgroup per problem
    "gm_spec":          (128, "gm", "fwd", "nearest", "fgrad", True, True, 0, "GM_SPEC", "latency", 0),
    "gm_spec_h":        (1, "gm", "fwd", "nearest", "fgrad", True, True, 0, "GM_SPEC_H", "latency", 0),
    # ... at 512 points per problem (the compile-time carve, fp32 only; N_512 points)
    "gm_spec_512":      (128, "gm", "fwd", "nearest", "fgrad", True, True, 0, "GM_SPEC_512", "latency", 0),
    "gm_spec_h_512":    (1, "gm", "fwd", "nearest", "fgrad", True, True, 0, "GM_SPEC_H_512", "latency", 0),
    "nearest_spec":     (128, "cauchy", "fwd", "nearest", "fgrad", True, True, 0, "NEAREST_SPEC", "latency", 0),
    "nearest_spec_h":   (1, "cauchy", "fwd", "nearest", "fgrad", True, True, 0, "NEAREST_SPEC_H", "latency", 0),
    "gm":               (128, "gm", "fwd", "nearest", "fgrad", True, False, 0, "GM", "latency", 0),
    "gm_h":             (1, "gm", "fwd", "nearest", "fgrad", True, False, 0, "GM_H", "latency", 0),
    "nearest":          (128, "cauchy", "fwd", "nearest", "fgrad", True, False, 0, "NEAREST", "latency", 0),
    "nearest_h":        (1, "cauchy", "fwd", "nearest", "fgrad", True, False, 0, "NEAREST_H", "latency", 0),
    # (compute_cost is one all-points evaluation: the planner keeps the team spread at B=1)
    "compute_cost":     (1, "gm", "cost", "nearest", "fgrad", True, True, 0, "NEAREST", "latency", 1),
    "bil_direct":       (1, "gm", "fwd", "bilinear", "fgrad", False, False, 1, "BIL_DIRECT", "latency", 0),
    "f_gm":             (1, "gm", "fwd", "nearest", "f", True, True, 1, "F_GM", "latency", 0),
    "f_nearest":        (1, "cauchy", "fwd", "nearest", "f", True, True, 1, "F_NEAREST", "latency", 0),
    # latency build, teams of workgroups
    "gm_team":          (1, "gm", "fwd", "nearest", "fgrad", True, True, 2, "GM", "latency", 1),
    "nearest_team":     (1, "cauchy", "fwd", "nearest", "fgrad", True, True, 2, "NEAREST", "latency", 1),
    "bil_direct_team":  (1, "gm", "fwd", "bilinear", "fgrad", False, False, 0, "BIL_DIRECT", "latency", 1),
    "f_gm_team":        (1, "gm", "fwd", "nearest", "f", True, True, 0, "F_GM", "latency", 1),
    "f_nearest_team":   (1, "cauchy", "fwd", "nearest", "f", True, True, 0, "F_NEAREST", "latency", 1),
    # throughput build (>= 2 problems per CU)
    "tp_gm":            (512, "gm", "fwd", "nearest", "fgrad", True, True, 0, "GM", "throughput", 0),
    "tp_nearest":       (512, "cauchy", "fwd", "nearest", "fgrad", True, True, 0, "NEAREST", "throughput", 0),
    "tp_bil_direct":    (512, "gm", "fwd", "bilinear", "fgrad", False, False, 0, "BIL_DIRECT", "throughput", 0),
    # wide build: the bilinear cell memo
    "bil_memo":         (128, "gm", "fwd", "bilinear", "fgrad", True, True, 0, "BILINEAR", "wide", 0),
    "bil_memo_team":    (1, "gm", "fwd", "bilinear", "fgrad", True, True, 0, "BILINEAR", "wide", 1),
}


def _cases():
    out = []
    for name, r in RECIPES.items():
        for dt in ("f32", "f64"):
            if (r[4] == "f" or name in M512) and dt == "f64":
                continue
            for ratio in (None, 0.8):
                out.append((name, dt, ratio))
    return out


CASES = _cases()


def case_key(name, dt, ratio):
    r = RECIPES[name]
    return (dt, r[9], r[10], int(ratio is not None), r[8])


def info_key(info):
    return (info["dtype_name"], info["build_name"], int(info["team"]), int(info["ratio"]), info["variant_name"])


_INPUTS = {}


def _inputs(seed, n_pts=N_PTS):
    """Device inputs of synthetic query `seed` (cached: cases share them)."""
    if (seed, n_pts) not in _INPUTS:
        init = "hard" if seed % 2 else "easy"
        _INPUTS[(seed, n_pts)] = synth.problem_inputs(n_pts, C, HF, WF, seed=1000 + seed, device=DEV, init=init)
    return _INPUTS[(seed, n_pts)]


_PACKED = {}


def _problem(seed, dt, layout, n_pts=N_PTS):
    key = (seed, dt, layout, n_pts)
    if key not in _PACKED:
        inp = _inputs(seed, n_pts)
        storage = torch.float64 if dt == "f64" else torch.float32
        fm = inp["fmap"].to(storage)
        feats = rf.pack_features(fm, storage=storage, device=DEV, layout=layout)
        _PACKED[key] = rf.make_problem(feats, inp["fref"].to(storage), inp["pts3d"], inp["K"], inp["im_width"],
                                       inp["im_height"], inp["R0"], inp["t0"])
    return _PACKED[key]


def _oracle(seed, loss_name, ratio, sampling, mode, n_pts=N_PTS):
    inp = _inputs(seed, n_pts)
    fm = inp["fmap"].double().cpu().numpy()
    gx, gy = orc.sobel(fm)
    fref = inp["fref"].double().cpu().numpy()
    if mode == "cost":
        return orc.compute_cost(inp["pts3d"], fref, fm, inp["K"], inp["im_width"], inp["im_height"], inp["R0"],
                                inp["t0"], ratio), None
    p = orc.make_problem(inp["pts3d"], fref, fm, gx, gy, inp["K"], inp["im_width"], inp["im_height"], inp["R0"],
                         inp["t0"])
    return orc.forward(p, orc.make_options(ITERS, 0.01, loss_name, ratio, sampling=sampling), trace_cap=ITERS + 1)


def rot_angle(Ra, Rb):
    c = (np.trace(np.asarray(Ra).T @ np.asarray(Rb)) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


@pytest.mark.parametrize("name,dt,ratio", CASES, ids=[f"{n}-{d}-{'r08' if r else 'nor'}" for n, d, r in CASES])
def test_specialisation_against_oracle(name, dt, ratio):
    B, loss, mode, sampling, layout, memo, spec, wgs, *_ = RECIPES[name]
    code, loss_name = LOSSES[loss]
    n_pts = N_512 if name in M512 else N_PTS
    probs = [_problem(q, dt, layout, n_pts) for q in range(B)]
    opts = rf.make_options(ITERS, 0.01, code, ratio_threshold=ratio, dtype=_lib.F64 if dt == "f64" else _lib.F32,
                           mode=_lib.MODE_COMPUTE_COST if mode == "cost" else _lib.MODE_FORWARD,
                           wgs_per_problem=wgs, memoize=memo, sampling=sampling, speculate=spec)
    res, trs = rf.refine(probs, opts, trace=mode == "fwd")
    info = _lib.last_launch()
    assert info_key(info) == case_key(name, dt, ratio), info
    subset = sorted({0, B // 2, B - 1})
    for q in subset:
        ores, otr = _oracle(q, loss_name, ratio, sampling, mode, n_pts)
        r = res[q]
        what = f"{name} {dt} ratio={ratio} query {q}"
        if mode == "cost":
            assert r["initial_cost"] == pytest.approx(ores, rel=1e-10 if dt == "f64" else 1e-6), what
            continue
        tr = trs[q]
        assert r["status"] & ~_lib.STATUS_HELPER_WAIT == 0, what
        assert r["n_evals"] == ores["n_evals"] and r["n_steps"] == ores["n_steps"], what
        np.testing.assert_array_equal(tr["n_supported"], otr["n_supported"], err_msg=what)
        if dt == "f64":
            np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-10, err_msg=what)
            np.testing.assert_allclose(r["R"], ores["R"], atol=1e-9, err_msg=what)
            np.testing.assert_allclose(r["t"], ores["t"], atol=1e-9, err_msg=what)
        else:
            np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-6, err_msg=what)
            assert rot_angle(r["R"], ores["R"]) < 1e-4, what
            assert np.linalg.norm(r["t"] - ores["t"]) < 1e-4, what
        assert r["best_num_inliers"] == ores["best_num_inliers"], what


def _sweep():
    """Every specialisation fmpnp_plan chooses over the grid (no launch)."""
    seen = {}
    grid = itertools.product(("f32", "f64"), ("fgrad", "f"), ("nearest", "bilinear"), ("gm", "cauchy"),
                             ("fwd", "cost"), (0, 1, 2), (None, 0.8), (1, 8, 128, 256, 512),
                             (64, 128, 480, 2048), (16, 512), (0, 2), (0, -1))
    for dt, layout, sampling, loss, mode, no_memo, ratio, B, N, Cc, wgs, helpers in grid:
        if layout == "f" and (dt == "f64" or sampling != "nearest"):
            continue
        desc = np.zeros(B, dtype=rf.PROBLEM_DTYPE)
        desc["feat"], desc["fref"], desc["pts3d"] = 256, 256, 256  # never dereferenced by the planner
        desc["Hf"], desc["Wf"], desc["cstride"], desc["c_end"], desc["ld_ref"] = HF, WF, Cc, Cc, Cc
        desc["N"], desc["im_width"], desc["im_height"] = N, 4 * WF, 4 * HF
        o = rf.make_options(ITERS, 0.01, LOSSES[loss][0], ratio_threshold=ratio,
                            dtype=_lib.F64 if dt == "f64" else _lib.F32,
                            mode=_lib.MODE_COMPUTE_COST if mode == "cost" else _lib.MODE_FORWARD,
                            wgs_per_problem=wgs, sampling=sampling, helpers=helpers)
        o.no_memo = no_memo
        o.layout = _lib.LAYOUT_F if layout == "f" else _lib.LAYOUT_FGRAD
        import ctypes
        info = _lib.LaunchInfo()
        rc = _lib.load().fmpnp_plan(desc.ctypes.data_as(ctypes.POINTER(_lib.Problem)), B, ctypes.byref(o),
                                    ctypes.byref(info))
        if rc == -4:  # FMPNP_ETOOBIG (e.g. the bilinear memo past its LDS)
            continue
        assert rc == 0, (dt, layout, sampling, loss, mode, no_memo, ratio, B, N, Cc, wgs, helpers, rc)
        seen.setdefault(info_key(_lib._info_dict(info)), (dt, layout, sampling, loss, mode, no_memo, ratio, B, N,
                                                          Cc, wgs, helpers))
    return seen


def test_every_planner_choice_has_an_oracle_case():
    seen = _sweep()
    covered = {case_key(*c) for c in CASES}
    missing = {k: v for k, v in seen.items() if k not in covered}
    assert not missing, f"specialisations the planner chooses without an oracle-compared case: {missing}"
    unreachable = covered - set(seen)
    assert not unreachable, f"cases for specialisations the sweep never chose: {sorted(unreachable)}"
