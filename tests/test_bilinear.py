"""Bilinear sampling (FMPNP_BILINEAR) -- an EXTENSION: the reference samples the nearest
texel only (featurePnP/model.py:74-97), so there is no reference output to pin it to
("parity unpinned").  Its definition (fmpnp_device.h bilinear_taps = oracle/fmpnp_oracle.c
bilinear_taps) is checked here three ways:
  * CPU: the oracle's first-evaluation cost equals an independent numpy restatement;
  * CPU: on a map that is affine in (x, y) the sampled features are exact, so the oracle's
    cost at the identity pose matches the closed form;
  * GPU: the HIP kernel follows the oracle's per-evaluation costs, steps and poses (fp64
    storage: 1e-10 / 1e-9; fp32 storage: the north-star 1e-4), independent of G.
"""
import math

import numpy as np
import pytest

import oracle.oracle as orc
from golden_io import case, maps64


def np_bilinear_cost(inp, f, R, t):
    """Mean 0.5||e||^2 with bilinear taps: plain numpy, no shared code with the oracle."""
    X = np.asarray(inp["pts3d"], np.float64).reshape(-1, 3)
    K = np.asarray(inp["K"], np.float64).reshape(3, 3)
    W, H = int(inp["im_width"]), int(inp["im_height"])
    C, Hf, Wf = f.shape
    fref = np.asarray(inp["fref"], np.float64)
    costs = []
    for n in range(X.shape[0]):
        P = [((R[i, 0] * X[n, 0] + R[i, 1] * X[n, 1]) + R[i, 2] * X[n, 2]) + t[i] for i in range(3)]
        u = [(K[i, 0] * P[0] + K[i, 1] * P[1]) + K[i, 2] * P[2] for i in range(3)]
        qx, qy = u[0] / u[2], u[1] / u[2]
        px, py = np.rint(qx) - 1.0, np.rint(qy) - 1.0
        if not (0 <= px < W and 0 <= py < H):
            continue
        sx = ((qx - 0.5) * Wf) / W - 0.5
        sy = ((qy - 0.5) * Hf) / H - 0.5
        x0, y0 = math.floor(sx), math.floor(sy)
        ax, ay = sx - x0, sy - y0
        cx = [min(max(x0, 0), Wf - 1), min(max(x0 + 1, 0), Wf - 1)]
        cy = [min(max(y0, 0), Hf - 1), min(max(y0 + 1, 0), Hf - 1)]
        v = ((1 - ax) * (1 - ay) * f[:, cy[0], cx[0]] + ax * (1 - ay) * f[:, cy[0], cx[1]]
             + (1 - ax) * ay * f[:, cy[1], cx[0]] + ax * ay * f[:, cy[1], cx[1]])
        e = v - fref[n, :C]
        costs.append(0.5 * float(e @ e))
    return float(np.mean(costs)) if costs else float("nan")


def oracle_problem(inp, f, gx, gy):
    return orc.make_problem(inp["pts3d"], inp["fref"], f, gx, gy, inp["K"], inp["im_width"], inp["im_height"],
                            inp["R0"], inp["t0"])


@pytest.mark.parametrize("name", ["gm_c16", "odd_geom_gm", "behind_camera_gm"])
def test_oracle_bilinear_initial_cost_matches_numpy(name):
    inp, meta, _ = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    p = oracle_problem(inp, f, gx, gy)
    res, tr = orc.forward(p, orc.make_options(1, 0.01, "squared", sampling="bilinear"), 8)
    want = np_bilinear_cost(inp, f, np.asarray(inp["R0"]).reshape(3, 3), np.asarray(inp["t0"]))
    assert tr["cost"][0] == pytest.approx(want, rel=1e-12)
    # and it is not the nearest-texel cost (the sampling really changed)
    res_nn, tr_nn = orc.forward(p, orc.make_options(1, 0.01, "squared"), 8)
    assert tr_nn["n_supported"][0] == tr["n_supported"][0]
    assert abs(tr_nn["cost"][0] - tr["cost"][0]) > 1e-9 * abs(tr["cost"][0])


def test_oracle_bilinear_exact_on_affine_map():
    """f_c(x, y) = a_c x + b_c y + d_c at texel (x, y): bilinear taps reproduce it exactly
    inside the map, so with fref = the affine value at each point's continuous texel
    coordinate the cost is zero (to rounding)."""
    rng = np.random.default_rng(3)
    C, Hf, Wf = 4, 40, 50
    W, H = 4 * Wf, 4 * Hf
    a, b, d = rng.normal(size=C), rng.normal(size=C), rng.normal(size=C)
    yy, xx = np.meshgrid(np.arange(Hf, dtype=np.float64), np.arange(Wf, dtype=np.float64), indexing="ij")
    f = a[:, None, None] * xx + b[:, None, None] * yy + d[:, None, None]
    gx, gy = orc.sobel(f)
    K = np.array([[0.8 * W, 0, W / 2], [0, 0.8 * W, H / 2], [0, 0, 1.0]])
    N = 64
    u = rng.uniform(0.2, 0.8, N) * W
    v = rng.uniform(0.2, 0.8, N) * H
    z = rng.uniform(5, 10, N)
    X = np.stack([(u - K[0, 2]) * z / K[0, 0], (v - K[1, 2]) * z / K[1, 1], z], 1)
    sx = ((u - 0.5) * Wf) / W - 0.5
    sy = ((v - 0.5) * Hf) / H - 0.5
    fref = a[None, :] * sx[:, None] + b[None, :] * sy[:, None] + d[None, :]
    p = orc.make_problem(X, fref, f, gx, gy, K, W, H, np.eye(3), np.zeros(3))
    _, tr = orc.forward(p, orc.make_options(1, 0.01, "squared", sampling="bilinear"), 4)
    assert tr["n_supported"][0] == N
    assert tr["cost"][0] < 1e-18


gpu = pytest.mark.gpu


def _gpu_case(name, storage, wgs=0, n_iters=None):
    import torch
    from fmpnp import _lib, refine as rf
    inp, meta, _ = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    feats = rf.pack_features(torch.from_numpy(f).to(storage), torch.from_numpy(gx).to(storage),
                             torch.from_numpy(gy).to(storage), storage=storage, device="cuda:0")
    prob = rf.make_problem(feats, torch.from_numpy(inp["fref"]), inp["pts3d"], inp["K"], inp["im_width"],
                           inp["im_height"], inp["R0"], inp["t0"])
    loss = {"geman_mcclure": _lib.GEMAN_MCCLURE, "cauchy": _lib.CAUCHY, "squared": _lib.SQUARED}[meta["loss"]]
    iters = n_iters or meta["n_iters"]
    opts = rf.make_options(iters, meta["lambda0"], loss, 0.0, meta.get("ratio_threshold"), feats.dtype_code,
                           wgs_per_problem=wgs, sampling="bilinear")
    (res,), tr = rf.refine([prob], opts, trace=True)
    p = oracle_problem(inp, f, gx, gy)
    ores, otr = orc.forward(p, orc.make_options(iters, meta["lambda0"], meta["loss"], meta.get("ratio_threshold"),
                                                sampling="bilinear"), 2 * iters + 2)
    return res, tr[0], ores, otr


@gpu
@pytest.mark.parametrize("name", ["gm_c16", "cauchy_c16", "ratio08_gm", "odd_geom_gm"])
def test_bilinear_fp64_follows_oracle(name):
    import torch
    res, tr, ores, otr = _gpu_case(name, torch.float64)
    n = len(otr["cost"])
    assert len(tr["cost"]) == n
    np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-10, atol=0)
    np.testing.assert_array_equal(tr["n_supported"], otr["n_supported"])
    np.testing.assert_allclose(tr["R"], otr["R"], atol=1e-9)
    np.testing.assert_allclose(res["R"], ores["R"], atol=1e-9)
    np.testing.assert_allclose(res["t"], ores["t"], atol=1e-9)
    assert res["best_cost"] == pytest.approx(ores["best_cost"], rel=1e-10)


@gpu
@pytest.mark.parametrize("name", ["gm_c16", "odd_geom_gm"])
def test_bilinear_fp32_within_north_star_tolerance(name):
    import torch
    res, _, ores, _ = _gpu_case(name, torch.float32)
    c = (np.trace(res["R"].T @ ores["R"]) - 1.0) / 2.0
    assert math.acos(max(-1.0, min(1.0, c))) < 1e-4
    assert np.linalg.norm(res["t"] - ores["t"]) < 1e-4


@gpu
def test_bilinear_independent_of_workgroups_per_problem():
    import torch
    base = _gpu_case("gm_c16", torch.float64, wgs=1)[0]
    for g in (2, 4):
        r = _gpu_case("gm_c16", torch.float64, wgs=g)[0]
        assert np.array_equal(r["R"], base["R"]) and np.array_equal(r["t"], base["t"])


# ---------------------------------------------------------------------------
# The cell memo (fmpnp_lm_impl.h eval_pass_bil): the default bilinear path keeps each point's
# 54 Bernstein coefficients per 2x2 cell and re-forms the six channel sums from them while the
# point stays in its cell; no_memo = 1 (VAR_BIL_DIRECT) samples every point at every evaluation.
# The two are the same sums up to fp64 rounding, so the fp64 tolerances of the oracle tests hold.
# ---------------------------------------------------------------------------
def _gpu_run(prob, iters, lambda0, loss, ratio, dtype_code, memo, wgs=0):
    from fmpnp import refine as rf
    opts = rf.make_options(iters, lambda0, loss, 0.0, ratio, dtype_code, wgs_per_problem=wgs, sampling="bilinear",
                           memoize=memo)
    (res,), (tr,) = rf.refine([prob], opts, trace=True)
    return res, tr


@gpu
@pytest.mark.parametrize("name", ["gm_c16", "cauchy_c16", "ratio08_gm", "odd_geom_gm", "behind_camera_gm"])
def test_bilinear_memo_matches_direct_sampling(name):
    import torch
    from fmpnp import _lib, refine as rf
    inp, meta, _ = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    feats = rf.pack_features(torch.from_numpy(f), torch.from_numpy(gx), torch.from_numpy(gy), storage=torch.float64,
                             device="cuda:0")
    prob = rf.make_problem(feats, torch.from_numpy(inp["fref"]), inp["pts3d"], inp["K"], inp["im_width"],
                           inp["im_height"], inp["R0"], inp["t0"])
    loss = {"geman_mcclure": _lib.GEMAN_MCCLURE, "cauchy": _lib.CAUCHY, "squared": _lib.SQUARED}[meta["loss"]]
    args = (prob, meta["n_iters"], meta["lambda0"], loss, meta.get("ratio_threshold"), feats.dtype_code)
    a, ta = _gpu_run(*args, memo=True)
    b, tb = _gpu_run(*args, memo=False)
    assert a["status"] == b["status"] and a["n_evals"] == b["n_evals"]
    np.testing.assert_array_equal(ta["n_supported"], tb["n_supported"])
    np.testing.assert_allclose(ta["cost"], tb["cost"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(a["R"], b["R"], atol=1e-11)
    np.testing.assert_allclose(a["t"], b["t"], atol=1e-11)
    # the memo gathers a cell once; direct sampling reads every supported point every evaluation
    assert a["texel_gathers"] <= b["texel_gathers"]


def _synthetic_bilinear(N, C, Hf, Wf, seed, init, c_begin=0, c_end=None, iters=50, wgs=0, memo=True):
    """fp32 packed maps of a synthetic query, the GPU bilinear run, and the oracle's run of
    the same inputs (fp64 CHW maps = the fp32 map exactly, fp64 Sobel)."""
    import torch
    from fmpnp import _lib, refine as rf, synth
    inp = synth.problem_inputs(N, C, Hf, Wf, seed=seed, device="cuda:0", init=init)
    feats = rf.pack_features(inp["fmap"], storage=torch.float32, device="cuda:0")
    prob = rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                           inp["R0"], inp["t0"], c_begin=c_begin, c_end=c_end)
    res, tr = _gpu_run(prob, iters, 0.01, _lib.GEMAN_MCCLURE, None, _lib.F32, memo, wgs)
    fm = inp["fmap"].double().cpu().numpy()
    gx, gy = orc.sobel(fm)
    p = orc.make_problem(inp["pts3d"], inp["fref"].double().cpu().numpy(), fm, gx, gy, inp["K"], inp["im_width"],
                         inp["im_height"], inp["R0"], inp["t0"], c_begin=c_begin, c_end=c_end)
    ores, otr = orc.forward(p, orc.make_options(iters, 0.01, "geman_mcclure", sampling="bilinear"), iters + 1)
    return res, tr, ores, otr


def _rot(Ra, Rb):
    c = (np.trace(np.asarray(Ra).T @ np.asarray(Rb)) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


@gpu
@pytest.mark.parametrize("shape,init,slc", [((512, 256, 240, 320), "easy", None),
                                            ((512, 256, 240, 320), "hard", None),
                                            ((256, 512, 60, 80), "hard", None),
                                            ((300, 256, 60, 80), "hard", (1, 203))])
def test_bilinear_memo_50_iters_against_oracle(shape, init, slc):
    """The bench's bilinear leg (cfg2 shape, fp32 texels, memo) for the full 50 iterations
    against the oracle's bilinear restatement; C = 512 takes the memo build's multi-round
    path, an unaligned channel slice its scalar path.  North-star tolerance on the pose,
    identical per-evaluation support counts, costs within 1e-6 (fp32 packed gradients)."""
    N, C, Hf, Wf = shape
    cb, ce = slc if slc else (0, None)
    res, tr, ores, otr = _synthetic_bilinear(N, C, Hf, Wf, seed=7, init=init, c_begin=cb, c_end=ce)
    assert res["status"] == 0 and res["n_evals"] == ores["n_evals"]
    np.testing.assert_array_equal(tr["n_supported"], otr["n_supported"])
    np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-6)
    assert _rot(res["R"], ores["R"]) < 1e-4
    assert np.linalg.norm(res["t"] - ores["t"]) < 1e-4
    # cells are re-gathered only when a point changes cell
    assert res["texel_gathers"] < 0.5 * N * res["n_evals"]
