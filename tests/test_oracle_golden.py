"""Pin the CPU oracle (oracle/) against the reference's own outputs (tests/golden/).

These run on CPU (no GPU marker).  The golden vectors were produced by the
reference implementation itself (tests/golden/gen_golden.py); the oracle is the
checker that the HIP path is compared against in test_gpu_parity.py.
"""
import math

import numpy as np
import pytest

import oracle.oracle as orc
from golden_io import ADAPTER_CASES, FORWARD_CASES, PYRAMID_CASES, case, load_npz, maps64, shared_fmap

# tolerances of the CPU restatement against torch (summation order differs in the last bits)
COST_RTOL = 1e-11
POSE_ATOL = 1e-10


def _accepts(costs):
    """accept/reject sequence from the tracked costs (model.py:469-486)."""
    acc, prev = [], costs[0]
    for c in costs[1:]:
        a = not (c > prev)
        acc.append(a)
        if a:
            prev = c
    return acc


def run_oracle_forward(name, trace_cap=256):
    inp, meta, gold = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    p = orc.make_problem(inp["pts3d"], inp["fref"], f, gx, gy, inp["K"], inp["im_width"], inp["im_height"],
                         inp["R0"], inp["t0"])
    o = orc.make_options(meta["n_iters"], meta["lambda0"], meta["loss"], meta.get("ratio_threshold"),
                         meta.get("barron_alpha"))
    res, tr = orc.forward(p, o, trace_cap)
    return inp, meta, gold, res, tr


def test_sobel_matches_reference():
    z = load_npz("sobel_small")
    gx, gy = orc.sobel(z["x"])
    np.testing.assert_allclose(gx, z["gx"], rtol=0, atol=1e-13)
    np.testing.assert_allclose(gy, z["gy"], rtol=0, atol=1e-13)


def test_sobel_shared_map_exact():
    z = load_npz("fmap_c16")
    gx, gy = orc.sobel(z["fmap32"].astype(np.float64))
    # sums of fp32 values with weights +-1, +-2 are exact in fp64: bit-equal probes
    assert np.array_equal(gx[:, ::7, ::9], z["gx_probe"])
    assert np.array_equal(gy[:, ::7, ::9], z["gy_probe"])
    assert gx.sum() == pytest.approx(float(z["gx_sum"]), rel=1e-12, abs=1e-12)


def test_kat_toy6_costs_exact():
    """Notebook KAT (FeatureBA_ToyExample.ipynb:477-478): 27497.41105769231 -> 276.125."""
    _, _, gold, res, tr = run_oracle_forward("kat_toy6")
    assert tr["cost"][0] == 27497.41105769231
    assert tr["cost"][-1] == 276.125
    assert len(tr["cost"]) == 51


@pytest.mark.parametrize("name", FORWARD_CASES)
def test_oracle_forward_matches_golden(name):
    inp, meta, gold, res, tr = run_oracle_forward(name)
    assert res["n_steps"] == int(gold["rec_n"])
    if "track_costs" in gold:
        gc = gold["track_costs"]
        assert len(tr["cost"]) == len(gc)
        np.testing.assert_allclose(tr["cost"], gc, rtol=COST_RTOL, atol=0)
        assert _accepts(list(tr["cost"])) == _accepts(list(gc))
        np.testing.assert_array_equal(tr["n_supported"], gold["track_npts"])
        np.testing.assert_allclose(tr["R"], gold["track_R"], rtol=0, atol=POSE_ATOL)
        np.testing.assert_allclose(tr["t"], gold["track_t"], rtol=0, atol=POSE_ATOL)
    else:
        assert len(tr["cost"]) == 0
    if int(gold["rec_n"]):
        sH = np.abs(gold["rec_H"]).max(axis=(1, 2), keepdims=True)
        np.testing.assert_allclose(tr["H"] / sH, gold["rec_H"] / sH, rtol=0, atol=1e-12)
        sg = np.abs(gold["rec_g"]).max(axis=1, keepdims=True)
        np.testing.assert_allclose(tr["g"] / sg, gold["rec_g"] / sg, rtol=0, atol=1e-12)
        np.testing.assert_array_equal(tr["lam"], gold["rec_lam"])
        np.testing.assert_array_equal(tr["lr"], gold["rec_lr"])
        sd = np.abs(gold["rec_delta"]).max(axis=1, keepdims=True)
        np.testing.assert_allclose(tr["delta"] / sd, gold["rec_delta"] / sd, rtol=0, atol=1e-9)
    np.testing.assert_allclose(res["R"], gold["out_R"], rtol=0, atol=POSE_ATOL)
    np.testing.assert_allclose(res["t"], gold["out_t"], rtol=0, atol=POSE_ATOL)
    assert res["has_best"] == bool(gold["has_best_cost_"])
    if res["has_best"]:
        assert res["best_cost"] == pytest.approx(float(gold["best_cost_"]), rel=COST_RTOL)
        assert res["best_num_inliers"] == int(gold["best_num_inliers_"])
        assert res["initial_cost"] == pytest.approx(float(gold["initial_cost_"]), rel=COST_RTOL)


def test_status_of_early_exits():
    *_, res, _ = run_oracle_forward("no_support_init")
    assert res["status"] == "no_support"
    *_, res, _ = run_oracle_forward("no_support_trial")
    assert res["status"] == "no_support_trial"


@pytest.mark.parametrize("name", PYRAMID_CASES)
def test_oracle_multilevel_matches_golden(name):
    inp, meta, gold = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    R, t, attrs, traces = orc.multilevel(meta["pyramid"], inp["pts3d"], inp["fref"], f, gx, gy, inp["K"],
                                         inp["im_width"], inp["im_height"], inp["R0"], inp["t0"],
                                         meta["n_iters"], meta["lambda0"], meta["loss"],
                                         meta.get("ratio_threshold"), meta.get("barron_alpha"), trace_cap=256)
    costs = np.concatenate([tr["cost"] for _, tr in traces])
    np.testing.assert_allclose(costs, gold["track_costs"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(R, gold["out_R"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(t, gold["out_t"], rtol=0, atol=1e-9)
    assert attrs["initial_cost"] == pytest.approx(float(gold["initial_cost_"]), rel=1e-11)
    assert attrs["best_cost"] == pytest.approx(float(gold["best_cost_"]), rel=1e-10)
    assert attrs["best_num_inliers"] == int(gold["best_num_inliers_"])


def test_compute_cost_matches_golden():
    z = load_npz("compute_cost")
    f = shared_fmap("fmap_c16").astype(np.float64)
    poses = {"init": (z["in_R0"], z["in_t0"]), "ident": (np.eye(3), np.zeros(3)),
             "away": (np.eye(3), np.array([500.0, 0.0, 0.0]))}
    for thr in (None, 0.8):
        for tag, (R, t) in poses.items():
            v = orc.compute_cost(z["in_pts3d"], z["in_fref"], f, z["in_K"], int(z["in_im_width"]),
                                 int(z["in_im_height"]), R, t, thr)
            g = float(z[f"cost_{tag}_{thr}"])
            if math.isnan(g):
                assert math.isnan(v)
            else:
                assert v == pytest.approx(g, rel=1e-12)


def test_quaternion_matches_golden():
    z = load_npz("quaternion")
    for M, q in zip(z["M"], z["q"]):
        np.testing.assert_allclose(orc.matrix_quaternion(M), q, rtol=0, atol=1e-15)


@pytest.mark.parametrize("name", ADAPTER_CASES)
def test_oracle_adapter_matches_golden(name):
    """feature_pnp (optimize_feature_pnp.py:50-71) restated: fref gather + fp64 cast + Sobel + LM."""
    z = load_npz(name)
    import json
    meta = json.loads(str(z["meta"]))
    img = meta["image_shape"]
    fref = orc.gather_reference_features(z["in_ref"].astype(np.float64), z["in_reference_inliers"], img)
    f = z["in_query"].astype(np.float64)
    gx, gy = orc.sobel(f)
    R0, t0 = z["in_matrix"][:3, :3], z["in_matrix"][:3, 3]
    pts = z["in_points_3d"].reshape(-1, 3)
    if meta["pyramid"] is None:
        p = orc.make_problem(pts, fref, f, gx, gy, z["in_K"], img[0], img[1], R0, t0)
        o = orc.make_options(meta["n_iters"], meta["lambda0"], meta["loss"])
        res, tr = orc.forward(p, o, 64)
        R, t = res["R"], res["t"]
        np.testing.assert_allclose(tr["cost"], z["track_costs"], rtol=1e-11)
        assert res["best_num_inliers"] == int(z["best_num_inliers_"])
    else:
        R, t, attrs, _ = orc.multilevel(meta["pyramid"], pts, fref, f, gx, gy, z["in_K"], img[0], img[1], R0, t0,
                                        meta["n_iters"], meta["lambda0"], meta["loss"])
        assert attrs["best_num_inliers"] == int(z["best_num_inliers_"])
    np.testing.assert_allclose(R, z["out_R"], atol=1e-10)
    np.testing.assert_allclose(t, z["out_t"], atol=1e-10)
    T = np.eye(4)
    T[:3, :3] = R
    T[3, :3] = t
    np.testing.assert_allclose(orc.matrix_quaternion(T), z["opt_quat"], atol=1e-10)
    np.testing.assert_allclose(t, z["opt_t"], atol=1e-10)


FIND_INLIERS_LOSSES = ("squared", "geman_mcclure", "cauchy")


def test_oracle_find_inliers_matches_golden():
    """find_inliers (model.py:131-152): support, NN costs, loss, ratio mask -- every pose,
    loss and threshold of the fixture, mask for mask."""
    z = load_npz("find_inliers")
    f = shared_fmap("fmap_c16").astype(np.float64)
    for tag in ("init", "ident", "shift"):
        for loss in FIND_INLIERS_LOSSES:
            for thr in (0.8, 0.5):
                mask, cost, nsup = orc.find_inliers(z["in_pts3d"], z["in_fref"], f, z["in_K"], int(z["in_im_width"]),
                                                    int(z["in_im_height"]), z[f"in_R_{tag}"], z[f"in_t_{tag}"], thr,
                                                    loss)
                np.testing.assert_array_equal(mask, z[f"mask_{tag}_{loss}_{thr}"].astype(bool), err_msg=tag + loss)
                assert nsup > 0


def oracle_feature_pnp_multi(z, given):
    """optimize_feature_pnp.py:20-47 composed from the oracle's pieces (gather, Sobel, LM, find_inliers)."""
    import json
    meta = json.loads(str(z["meta"]))
    img = meta["image_shape"]
    fref = orc.gather_reference_features(z["in_ref"].astype(np.float64), z["in_reference_inliers"], img)
    f = z["in_query"].astype(np.float64)
    gx, gy = orc.sobel(f)
    pts = z["in_points_3d"].reshape(-1, 3)
    R, t = z["in_matrix"][:3, :3], z["in_matrix"][:3, 3]
    thr = meta["find_inliers_threshold"]
    if given:
        inl = np.zeros(len(pts), dtype=bool)
        inl[z["in_mask_given"]] = True
    else:
        inl = orc.find_inliers(pts, fref, f, z["in_K"], img[0], img[1], R, t, thr)[0]
    o = orc.make_options(meta["n_iters"], meta["lambda0"], meta["loss"])
    initial = None
    for _ in range(3):
        p = orc.make_problem(pts[inl], fref[inl], f, gx, gy, z["in_K"], img[0], img[1], R, t)
        res, _tr = orc.forward(p, o, 0)
        R, t = res["R"], res["t"]
        initial = res["initial_cost"] if initial is None else initial
        inl = orc.find_inliers(pts, fref, f, z["in_K"], img[0], img[1], R, t, thr)[0]
    return R, t, initial, res


@pytest.mark.parametrize("tag", ["none", "given"])
def test_oracle_feature_pnp_multi_matches_golden(tag):
    z = load_npz("feature_pnp_multi")
    R, t, initial, res = oracle_feature_pnp_multi(z, tag == "given")
    np.testing.assert_allclose(R, z[f"out_R_{tag}"], atol=POSE_ATOL)
    np.testing.assert_allclose(t, z[f"out_t_{tag}"], atol=POSE_ATOL)
    assert initial == pytest.approx(float(z[f"initial_cost_{tag}"]), rel=COST_RTOL)
    assert res["best_cost"] == pytest.approx(float(z[f"best_cost_{tag}"]), rel=COST_RTOL)
    assert res["best_num_inliers"] == int(z[f"best_num_inliers_{tag}"])


@pytest.mark.parametrize("name", ["ratio08_gm", "ratio05_sq"])
def test_oracle_ratio_masks_match_reference_track(name):
    """track_["threshold_mask"] of the reference's ratio-test runs: the oracle's find_inliers
    at each tracked pose, restricted to the supported points, is the reference's mask."""
    inp, meta, gold = case(name)
    f, _, _ = maps64(inp, orc.sobel)
    tm = load_npz(f"track_thr_{name}")["threshold_mask"]
    assert tm.shape[0] == len(gold["track_R"])
    for k in range(tm.shape[0]):
        mask, _, nsup = orc.find_inliers(inp["pts3d"], inp["fref"], f, inp["K"], int(inp["im_width"]),
                                         int(inp["im_height"]), gold["track_R"][k], gold["track_t"][k],
                                         meta["ratio_threshold"], meta["loss"])
        sup = tm[k] >= 0
        assert nsup == int(sup.sum())
        np.testing.assert_array_equal(mask[sup], tm[k][sup] == 1)
