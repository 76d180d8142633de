"""HIP path vs the reference's golden vectors and the CPU oracle (needs an MI355X).

Every test here calls the product path (libfmpnp.so through the fmpnp façade
or the C ABI); the oracle (oracle/) and the golden vectors are only the checkers.

Tolerances (stated per test):
  * fp64 texel storage: the trajectory is the reference's -- identical
    accept/reject sequence and per-evaluation support counts, costs to 1e-10
    relative, poses to 1e-9;
  * fp32 texel storage (the performance layout): final pose within 1e-4 rad /
    1e-4 m of the fp64 reference path after the same iteration count (north star).
"""
import math

import numpy as np
import pytest
import torch

import oracle.oracle as orc
from golden_io import ADAPTER_CASES, FORWARD_CASES, PYRAMID_CASES, case, load_npz, maps64, shared_fmap

pytestmark = pytest.mark.gpu

import fmpnp  # noqa: E402  (no skip: a missing HIP library must fail the GPU run)
from fmpnp import _lib, refine as rf, synth  # noqa: E402

DEV = "cuda:0"
LOSS = {"squared": _lib.SQUARED, "huber": _lib.HUBER, "cauchy": _lib.CAUCHY, "geman_mcclure": _lib.GEMAN_MCCLURE,
        "barron": _lib.BARRON}


def rot_angle(Ra, Rb):
    c = (np.trace(np.asarray(Ra).T @ np.asarray(Rb)) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


def accepts(costs):
    acc, prev = [], costs[0]
    for c in costs[1:]:
        a = not (c > prev)
        acc.append(a)
        if a:
            prev = c
    return acc


def run_case(name, storage=torch.float64, wgs=0, trace=True):
    inp, meta, gold = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    feats = rf.pack_features(torch.from_numpy(f).to(storage), torch.from_numpy(gx).to(storage),
                             torch.from_numpy(gy).to(storage), storage=storage, device=DEV)
    prob = rf.make_problem(feats, torch.from_numpy(inp["fref"]), inp["pts3d"], inp["K"], inp["im_width"],
                           inp["im_height"], inp["R0"], inp["t0"])
    opts = rf.make_options(meta["n_iters"], meta["lambda0"], LOSS[meta["loss"]], meta.get("barron_alpha") or 0.0,
                           meta.get("ratio_threshold"), feats.dtype_code, wgs_per_problem=wgs)
    (res,), tr = rf.refine([prob], opts, trace=trace)
    return inp, meta, gold, res, (tr[0] if tr else None)


@pytest.mark.parametrize("name", FORWARD_CASES)
def test_forward_fp64_matches_reference(name):
    inp, meta, gold, res, tr = run_case(name)
    assert res["n_steps"] == int(gold["rec_n"])
    if "track_costs" in gold:
        gc = gold["track_costs"]
        assert len(tr["cost"]) == len(gc)
        np.testing.assert_allclose(tr["cost"], gc, rtol=1e-10, atol=0)
        assert list(tr["accepted"][1:]) == accepts(list(gc))
        np.testing.assert_array_equal(tr["n_supported"], gold["track_npts"])
        np.testing.assert_allclose(tr["R"], gold["track_R"], atol=1e-9)
        np.testing.assert_allclose(tr["t"], gold["track_t"], atol=1e-9)
        m = min(len(gc), int(gold["rec_n"]))
        np.testing.assert_array_equal(tr["lam"][1:m], gold["rec_lam"][1:m])
        np.testing.assert_array_equal(tr["lr"][1:m], gold["rec_lr"][1:m])
    np.testing.assert_allclose(res["R"], gold["out_R"], atol=1e-9)
    np.testing.assert_allclose(res["t"], gold["out_t"], atol=1e-9)
    assert res["has_best"] == bool(gold["has_best_cost_"])
    if res["has_best"]:
        assert res["best_cost"] == pytest.approx(float(gold["best_cost_"]), rel=1e-10)
        assert res["best_num_inliers"] == int(gold["best_num_inliers_"])
        assert res["initial_cost"] == pytest.approx(float(gold["initial_cost_"]), rel=1e-10)


def test_kat_toy6_on_gpu():
    """FeatureBA_ToyExample.ipynb:477-478 on the device."""
    _, _, _, res, tr = run_case("kat_toy6")
    assert tr["cost"][0] == pytest.approx(27497.41105769231, rel=1e-13)
    assert tr["cost"][-1] == pytest.approx(276.125, rel=1e-13)
    assert len(tr["cost"]) == 51


def test_early_exit_status():
    *_, res, _ = run_case("no_support_init")
    assert res["status"] == _lib.STATUS_NO_SUPPORT and not res["has_best"]
    *_, res, _ = run_case("no_support_trial")
    assert res["status"] == _lib.STATUS_NO_SUPPORT_TRIAL


@pytest.mark.parametrize("name", ["gm_c16", "cauchy_c16", "ratio08_gm", "odd_geom_gm", "behind_camera_gm"])
def test_forward_fp32_within_north_star_tolerance(name):
    inp, meta, gold, res, _ = run_case(name, storage=torch.float32, trace=False)
    assert rot_angle(res["R"], gold["out_R"]) < 1e-4
    assert np.linalg.norm(res["t"] - gold["out_t"]) < 1e-4


@pytest.mark.parametrize("name", ["gm_c16", "ratio08_gm", "odd_geom_ratio_cauchy"])
def test_results_independent_of_workgroups_per_problem(name):
    """Chunk partials are summed in chunk order: G=1..8 give bit-identical results."""
    base = run_case(name, wgs=1)[3]
    for g in (2, 3, 8):
        r = run_case(name, wgs=g)[3]
        assert np.array_equal(r["R"], base["R"]) and np.array_equal(r["t"], base["t"])
        assert r["best_cost"] == base["best_cost"] or (math.isnan(r["best_cost"]) and math.isnan(base["best_cost"]))


def test_deterministic_repeat():
    a = run_case("gm_c16", storage=torch.float32)[3]
    b = run_case("gm_c16", storage=torch.float32)[3]
    assert np.array_equal(a["R"], b["R"]) and np.array_equal(a["t"], b["t"]) and a["best_cost"] == b["best_cost"]


def test_batch_equals_individual():
    """Different problems (different maps, N, losses are shared) in one launch."""
    names = ["gm_c16", "behind_camera_gm", "odd_geom_gm", "no_support_init"]
    probs, singles = [], []
    for nm in names:
        inp, meta, gold = case(nm)
        f, gx, gy = maps64(inp, orc.sobel)
        feats = rf.pack_features(torch.from_numpy(f), torch.from_numpy(gx), torch.from_numpy(gy),
                                 storage=torch.float64, device=DEV)
        probs.append(rf.make_problem(feats, torch.from_numpy(inp["fref"]), inp["pts3d"], inp["K"], inp["im_width"],
                                     inp["im_height"], inp["R0"], inp["t0"]))
    opts = rf.make_options(20, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F64)
    batch, _ = rf.refine(probs, opts)
    for p, rb in zip(probs, batch):
        (r1,), _ = rf.refine([p], opts)
        assert np.array_equal(r1["R"], rb["R"]) and np.array_equal(r1["t"], rb["t"])
        assert r1["status"] == rb["status"]


@pytest.mark.parametrize("wps", ["2", "4"])
def test_large_batch_throughput_variant_equals_individual(wps, monkeypatch):
    """n >= 2 x CUs: the problems run in rounds of resident teams (default) or, with
    FMPNP_LM_WPS=4, on the two-workgroups-per-CU kernel (128 VGPRs); either way the results
    must be bit-identical to single-problem launches (the 256-VGPR kernel)."""
    monkeypatch.setenv("FMPNP_LM_WPS", wps)
    names = ["gm_c16", "behind_camera_gm", "odd_geom_gm", "no_support_init", "ratio08_gm"]
    base = []
    for nm in names:
        inp, meta, gold = case(nm)
        f, gx, gy = maps64(inp, orc.sobel)
        feats = rf.pack_features(torch.from_numpy(f), torch.from_numpy(gx), torch.from_numpy(gy),
                                 storage=torch.float32, device=DEV)
        base.append(rf.make_problem(feats, torch.from_numpy(inp["fref"]), inp["pts3d"], inp["K"], inp["im_width"],
                                    inp["im_height"], inp["R0"], inp["t0"]))
    n = 2 * torch.cuda.get_device_properties(0).multi_processor_count + 3
    probs = [base[i % len(base)] for i in range(n)]
    opts = rf.make_options(20, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
    batch, _ = rf.refine(probs, opts)
    assert _lib.last_launch()["grid"] >= n
    singles = [rf.refine([p], opts)[0][0] for p in base]
    for i, rb in enumerate(batch):
        r1 = singles[i % len(base)]
        assert np.array_equal(r1["R"], rb["R"]) and np.array_equal(r1["t"], rb["t"]), i
        assert r1["status"] == rb["status"] and r1["n_evals"] == rb["n_evals"]


def test_pack_sobel_matches_oracle():
    z = load_npz("sobel_small")
    x = z["x"]
    feats = rf.pack_features(torch.from_numpy(x), storage=torch.float64, device=DEV)
    buf = feats.buf.cpu().numpy()  # [H][W][3][cs]
    C = x.shape[0]
    np.testing.assert_array_equal(buf[:, :, 0, :C].transpose(2, 0, 1), x)
    np.testing.assert_allclose(buf[:, :, 1, :C].transpose(2, 0, 1), z["gx"], atol=1e-13, rtol=0)
    np.testing.assert_allclose(buf[:, :, 2, :C].transpose(2, 0, 1), z["gy"], atol=1e-13, rtol=0)
    # fp32 hypercolumn: the fp64 Sobel of fp32 values is exact -> bit-equal to the oracle
    f32 = shared_fmap("fmap_c16")
    feats = rf.pack_features(torch.from_numpy(f32), storage=torch.float64, device=DEV)
    gx, gy = orc.sobel(f32.astype(np.float64))
    buf = feats.buf.cpu().numpy()
    assert np.array_equal(buf[:, :, 1, :16].transpose(2, 0, 1), gx)
    assert np.array_equal(buf[:, :, 2, :16].transpose(2, 0, 1), gy)


def test_pack_large_tiles_and_ragged_edges():
    """Maps larger than one 64x64x8 tile with ragged edges; fp32 in/out."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn((70, 37, 131), generator=g, dtype=torch.float32)
    feats = rf.pack_features(x, storage=torch.float32, device=DEV)
    gx, gy = orc.sobel(x.double().numpy())
    buf = feats.buf.cpu().numpy()
    assert feats.cstride == 72
    np.testing.assert_array_equal(buf[:, :, 0, :70].transpose(2, 0, 1), x.numpy())
    np.testing.assert_array_equal(buf[:, :, 1, :70].transpose(2, 0, 1), gx.astype(np.float32))
    np.testing.assert_array_equal(buf[:, :, 2, :70].transpose(2, 0, 1), gy.astype(np.float32))
    assert not buf[:, :, :, 70:].any()


def _sobel_np(x, normalized, replicate):
    """3x3 Sobel cross-correlation (helpers/sobel_pytorch.py:9-59) with zero or edge padding."""
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1)), mode="edge" if replicate else "constant")
    a, b, c2 = xp[:, :-2, :-2], xp[:, :-2, 1:-1], xp[:, :-2, 2:]
    d, e = xp[:, 1:-1, :-2], xp[:, 1:-1, 2:]
    g, h, k = xp[:, 2:, :-2], xp[:, 2:, 1:-1], xp[:, 2:, 2:]
    gx = ((-a + c2) + (-2.0 * d + 2.0 * e)) + (-g + k)
    gy = ((-a - 2.0 * b) - c2) + ((g + 2.0 * h) + k)
    s = 0.125 if normalized else 1.0
    return gx * s, gy * s


@pytest.mark.parametrize("shape,dtype,normalized,replicate", [
    ((256, 240, 320), torch.float32, False, False),   # cfg2: 16-B vector loads, full tiles
    ((130, 33, 100), torch.float32, True, True),      # partial channel block, W%32 != 0 (scalar edge tile)
    ((9, 17, 131), torch.float32, False, True),       # W*4 not 16-B aligned: scalar loads throughout
    ((70, 21, 66), torch.float64, True, False),       # fp64 input, 16-B (double2) vector loads
    ((3, 5, 7), torch.float64, False, True),          # fewer rows than one tile
])
def test_pack_sobel_variants(shape, dtype, normalized, replicate):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(shape, generator=g, dtype=dtype)
    storage = torch.float64 if dtype == torch.float64 else torch.float32
    feats = rf.pack_features(x, storage=storage, device=DEV, sobel_normalized=normalized,
                             sobel_replicate_pad=replicate)
    gx, gy = _sobel_np(x.double().numpy(), normalized, replicate)
    buf = feats.buf.cpu().numpy()
    C = shape[0]
    np.testing.assert_array_equal(buf[:, :, 0, :C].transpose(2, 0, 1), x.numpy())
    np.testing.assert_array_equal(buf[:, :, 1, :C].transpose(2, 0, 1), gx.astype(buf.dtype))
    np.testing.assert_array_equal(buf[:, :, 2, :C].transpose(2, 0, 1), gy.astype(buf.dtype))
    assert not buf[:, :, :, C:].any()
    if not normalized and not replicate and dtype == torch.float32:
        ogx, ogy = orc.sobel(x.double().numpy())
        assert np.array_equal(ogx, gx) and np.array_equal(ogy, gy)


def test_gather_reference_matches_oracle():
    z = load_npz("adapter_nonsquare")
    import json
    img = json.loads(str(z["meta"]))["image_shape"]
    ref = torch.from_numpy(z["in_ref"])
    got = rf.gather_reference(ref, z["in_reference_inliers"], img, storage=torch.float64, device=DEV)
    want = orc.gather_reference_features(z["in_ref"].astype(np.float64), z["in_reference_inliers"], img)
    np.testing.assert_array_equal(got.cpu().numpy()[:, :want.shape[1]], want)


@pytest.mark.parametrize("name", PYRAMID_CASES)
def test_multilevel_facade_matches_reference(name):
    inp, meta, gold = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    loss = fmpnp.losses.BY_NAME[meta["loss"]]
    m = fmpnp.sparseFeaturePnP(meta["n_iters"], loss_fn=loss, lambda_=meta["lambda0"],
                               ratio_threshold=meta.get("ratio_threshold"))
    R, t = m.multilevel_optimization([tuple(l) for l in meta["pyramid"]], torch.from_numpy(inp["pts3d"]),
                                     torch.from_numpy(inp["fref"]), torch.from_numpy(f), torch.from_numpy(gx),
                                     torch.from_numpy(gy), torch.from_numpy(inp["K"]), int(inp["im_width"]),
                                     int(inp["im_height"]), R_init=torch.from_numpy(inp["R0"]),
                                     t_init=torch.from_numpy(inp["t0"]), track=True)
    np.testing.assert_allclose(np.array(m.track_["costs"]), gold["track_costs"], rtol=1e-9)
    np.testing.assert_allclose(R.numpy(), gold["out_R"], atol=1e-8)
    np.testing.assert_allclose(t.numpy(), gold["out_t"], atol=1e-8)
    assert m.initial_cost_.item() == pytest.approx(float(gold["initial_cost_"]), rel=1e-10)
    assert m.best_cost_.item() == pytest.approx(float(gold["best_cost_"]), rel=1e-9)
    assert m.best_num_inliers_ == int(gold["best_num_inliers_"])


def test_forward_facade_track_matches_reference():
    inp, meta, gold = case("ratio08_gm")
    f, gx, gy = maps64(inp, orc.sobel)
    m = fmpnp.sparseFeaturePnP(meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss, lambda_=meta["lambda0"],
                               ratio_threshold=0.8)
    R, t = m(torch.from_numpy(inp["pts3d"]), torch.from_numpy(inp["fref"]), torch.from_numpy(f),
             torch.from_numpy(gx), torch.from_numpy(gy), torch.from_numpy(inp["K"]), int(inp["im_width"]),
             int(inp["im_height"]), R_init=torch.from_numpy(inp["R0"]), t_init=torch.from_numpy(inp["t0"]),
             track=True)
    assert R.dtype == torch.float64 and R.device.type == "cpu"
    np.testing.assert_allclose(np.array(m.track_["costs"]), gold["track_costs"], rtol=1e-10)
    np.testing.assert_array_equal(np.stack([p.numpy() for p in m.track_["points2d"]]), gold["track_points2d"])
    np.testing.assert_array_equal(np.stack([k.numpy() for k in m.track_["mask"]]).astype(np.int8),
                                  gold["track_mask"])
    assert m.best_num_inliers_ == int(gold["best_num_inliers_"])
    # threshold masks over the supported points (model.py:328,452), as the reference tracked them
    tm = load_npz("track_thr_ratio08_gm")["threshold_mask"]
    assert len(m.track_["threshold_mask"]) == tm.shape[0]
    for k, thm in enumerate(m.track_["threshold_mask"]):
        sup = tm[k] >= 0
        np.testing.assert_array_equal(thm.numpy(), tm[k][sup] == 1, err_msg=f"eval {k}")


def test_compute_cost_facade_matches_reference():
    z = load_npz("compute_cost")
    f = torch.from_numpy(shared_fmap("fmap_c16").astype(np.float64))
    for thr in (None, 0.8):
        m = fmpnp.sparseFeaturePnP(1, ratio_threshold=thr)
        for tag, (R, t) in {"init": (z["in_R0"], z["in_t0"]), "ident": (np.eye(3), np.zeros(3)),
                            "away": (np.eye(3), np.array([500.0, 0.0, 0.0]))}.items():
            v = m.compute_cost(torch.from_numpy(z["in_pts3d"]), torch.from_numpy(R), torch.from_numpy(t), f,
                               torch.from_numpy(z["in_fref"]), torch.from_numpy(z["in_K"]), int(z["in_im_width"]),
                               int(z["in_im_height"]))
            g = float(z[f"cost_{tag}_{thr}"])
            if tag == "away":  # no supported point: the reference returns None (model.py:226-227)
                assert v is None
            elif math.isnan(g):  # all residuals 0 -> ratio test keeps nothing -> mean of empty = NaN
                assert math.isnan(v.item())
            else:
                assert v.item() == pytest.approx(g, rel=1e-12)


@pytest.mark.parametrize("name", ADAPTER_CASES)
def test_adapter_feature_pnp_matches_reference(name):
    import json
    from collections import namedtuple
    z = load_npz(name)
    meta = json.loads(str(z["meta"]))
    Pred = namedtuple("Prediction", "points_3d reference_inliers matrix quaternion reference_filename")
    pred = Pred(z["in_points_3d"], z["in_reference_inliers"], z["in_matrix"], np.array([1.0, 0, 0, 0]), "ref.png")
    q = torch.from_numpy(z["in_query"]).to(DEV)[None]
    r = torch.from_numpy(z["in_ref"]).to(DEV)[None]
    model = fmpnp.sparseFeaturePnP(meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss, lambda_=meta["lambda0"],
                                   storage=torch.float64)
    pyr = [tuple(l) for l in meta["pyramid"]] if meta["pyramid"] else None
    R, t, model = fmpnp.feature_pnp(q, r, pred, z["in_K"], tuple(meta["image_shape"]), track=True,
                                    feature_pyramid=pyr, model=model)
    np.testing.assert_allclose(R.numpy(), z["out_R"], atol=1e-9)
    np.testing.assert_allclose(t.numpy(), z["out_t"], atol=1e-9)
    assert model.best_num_inliers_ == int(z["best_num_inliers_"])

    class Net:
        def compute_hypercolumn(self, names, to_cpu=False, resize=True):
            return r, None

    model2 = fmpnp.sparseFeaturePnP(meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss, lambda_=meta["lambda0"],
                                    storage=torch.float64)
    tl, ql, _ = fmpnp.optimize_feature_pnp(q, Net(), pred, z["in_K"], tuple(meta["image_shape"]),
                                           feature_pyramid=pyr, model=model2)
    np.testing.assert_allclose(np.array(ql), z["opt_quat"], atol=1e-9)
    np.testing.assert_allclose(np.array(tl), z["opt_t"], atol=1e-9)


def _oracle_on(inputs, n_iters, loss="geman_mcclure", ratio=None):
    fm = inputs["fmap"].double().cpu().numpy()
    gx, gy = orc.sobel(fm)
    p = orc.make_problem(inputs["pts3d"], inputs["fref"].double().cpu().numpy(), fm, gx, gy, inputs["K"],
                         inputs["im_width"], inputs["im_height"], inputs["R0"], inputs["t0"])
    return orc.forward(p, orc.make_options(n_iters, 0.01, loss, ratio), trace_cap=n_iters + 1)


@pytest.mark.parametrize("storage", [torch.float32, torch.float64])
def test_cfg2_shape_against_oracle(storage):
    """BASELINE config 2 shape (N=512, C=256, 240x320, GM), 8 iterations vs the oracle."""
    inputs = synth.problem_inputs(512, 256, 240, 320, seed=3, device=DEV)
    n_iters = 8
    ores, otr = _oracle_on(inputs, n_iters)
    feats = rf.pack_features(inputs["fmap"], storage=storage, device=DEV)
    prob = rf.make_problem(feats, inputs["fref"], inputs["pts3d"], inputs["K"], inputs["im_width"],
                           inputs["im_height"], inputs["R0"], inputs["t0"])
    (res,), (tr,) = rf.refine([prob], rf.make_options(n_iters, 0.01, _lib.GEMAN_MCCLURE, dtype=feats.dtype_code),
                              trace=True)
    assert rot_angle(res["R"], ores["R"]) < 1e-4
    assert np.linalg.norm(res["t"] - ores["t"]) < 1e-4
    np.testing.assert_array_equal(tr["n_supported"], otr["n_supported"])
    np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-9 if storage == torch.float64 else 1e-6)


@pytest.mark.parametrize("storage", [torch.float32, torch.float64])
def test_cfg5_shape_against_oracle(storage):
    """BASELINE config 5 shape (N=2048, C=512, 480x640, Cauchy, robotcar_inlier_GN.gin): C > 64 V
    takes the multi-round gather, and 2048 points exceed one workgroup's LDS (G >= 2)."""
    inputs = synth.problem_inputs(2048, 512, 480, 640, seed=5, device=DEV)
    n_iters = 5
    ores, otr = _oracle_on(inputs, n_iters, loss="cauchy")
    feats = rf.pack_features(inputs["fmap"], storage=storage, device=DEV)
    prob = rf.make_problem(feats, inputs["fref"], inputs["pts3d"], inputs["K"], inputs["im_width"],
                           inputs["im_height"], inputs["R0"], inputs["t0"])
    (res,), (tr,) = rf.refine([prob], rf.make_options(n_iters, 0.01, _lib.CAUCHY, dtype=feats.dtype_code),
                              trace=True)
    assert _lib.last_launch()["wgs_per_problem"] >= 2
    assert rot_angle(res["R"], ores["R"]) < 1e-4
    assert np.linalg.norm(res["t"] - ores["t"]) < 1e-4
    np.testing.assert_array_equal(tr["n_supported"], otr["n_supported"])
    np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-9 if storage == torch.float64 else 1e-6)
    del feats, prob


def test_batch_of_synthetic_queries_and_dtype_f32():
    """A batch of cfg2-like queries (smaller maps) against per-query oracle runs."""
    probs, ins = [], []
    for s in range(6):
        inp = synth.problem_inputs(200 + 37 * s, 64, 60, 80, seed=10 + s, device=DEV)
        feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=DEV)
        probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                     inp["R0"], inp["t0"]))
        ins.append(inp)
    res, _ = rf.refine(probs, rf.make_options(20, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32))
    for inp, r in zip(ins, res):
        o, _ = _oracle_on(inp, 20)
        assert rot_angle(r["R"], o["R"]) < 1e-4
        assert np.linalg.norm(r["t"] - o["t"]) < 1e-4


def test_async_batch_matches_sync():
    inputs = synth.problem_inputs(300, 64, 60, 80, seed=77, device=DEV)
    feats = rf.pack_features(inputs["fmap"], storage=torch.float32, device=DEV)
    prob = rf.make_problem(feats, inputs["fref"], inputs["pts3d"], inputs["K"], inputs["im_width"],
                           inputs["im_height"], inputs["R0"], inputs["t0"])
    opts = rf.make_options(15, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
    sync_r = rf.refine([prob], opts)[0][0]
    ab = rf.AsyncBatch([prob] * 3, opts)
    ab.launch()
    ab.launch()
    for r in ab.results():
        assert np.array_equal(r["R"], sync_r["R"]) and np.array_equal(r["t"], sync_r["t"])


@pytest.mark.parametrize("storage", [torch.float64, torch.float32])
def test_find_inliers_matches_reference(storage):
    """find_inliers (model.py:131-152) through fmpnp_point_costs: the reference's masks for
    every pose / loss / threshold of the fixture; per-point costs against the oracle's to
    1e-12 relative (summation order).  The C=16 map is fp32 data, so fp32 (f-only layout)
    and fp64 storage hold the same values and give the same masks."""
    z = load_npz("find_inliers")
    f = shared_fmap("fmap_c16").astype(np.float64)
    fm = torch.from_numpy(f).to(storage)
    W, H = int(z["in_im_width"]), int(z["in_im_height"])
    losses = {"squared": fmpnp.squared_loss, "geman_mcclure": fmpnp.geman_mcclure_loss,
              "cauchy": fmpnp.cauchy_loss}
    for tag in ("init", "ident", "shift"):
        R, t = z[f"in_R_{tag}"], z[f"in_t_{tag}"]
        for loss, fn in losses.items():
            for thr in (0.8, 0.5):
                m = fmpnp.find_inliers(torch.from_numpy(z["in_pts3d"]), torch.from_numpy(R), torch.from_numpy(t), fm,
                                       torch.from_numpy(z["in_fref"]), torch.from_numpy(z["in_K"]), W, H,
                                       threshold=thr, loss_fn=fn)
                assert m.dtype == torch.bool and m.device.type == "cpu"
                np.testing.assert_array_equal(m.numpy(), z[f"mask_{tag}_{loss}_{thr}"].astype(bool),
                                              err_msg=f"{tag} {loss} {thr}")
        feats = rf.pack_features(fm, storage=storage, device=DEV,
                                 layout="f" if storage == torch.float32 else "fgrad")
        prob = rf.make_problem(feats, z["in_fref"], z["in_pts3d"], z["in_K"], W, H, R, t)
        cost, sup = rf.point_costs(prob)
        _, ocost, nsup = orc.find_inliers(z["in_pts3d"], z["in_fref"], f, z["in_K"], W, H, R, t, 0.8)
        assert int(sup.sum()) == nsup
        np.testing.assert_allclose(cost.cpu().numpy(), ocost, rtol=1e-12, atol=0)


def test_find_inliers_reference_errors():
    """mode other than "ratio_max" -> None; no threshold -> TypeError (gin binds it in the
    reference); no supported point -> torch.max of an empty tensor raises."""
    z = load_npz("find_inliers")
    fm = torch.from_numpy(shared_fmap("fmap_c16").astype(np.float64))
    args = (torch.from_numpy(z["in_pts3d"]), torch.eye(3, dtype=torch.float64), torch.zeros(3, dtype=torch.float64),
            fm, torch.from_numpy(z["in_fref"]), torch.from_numpy(z["in_K"]), int(z["in_im_width"]),
            int(z["in_im_height"]))
    assert fmpnp.find_inliers(*args, threshold=0.8, mode="other") is None
    with pytest.raises(TypeError):
        fmpnp.find_inliers(*args)
    away = list(args)
    away[2] = torch.tensor([500.0, 0.0, 0.0], dtype=torch.float64)
    with pytest.raises(RuntimeError):
        fmpnp.find_inliers(*away, threshold=0.8)
    fmpnp.config.configure(find_inliers_threshold=0.8)
    try:
        assert fmpnp.find_inliers(*args).shape == (z["in_pts3d"].shape[0],)
    finally:
        fmpnp.config.configure(find_inliers_threshold=None)


@pytest.mark.parametrize("tag", ["none", "given"])
@pytest.mark.parametrize("storage", [torch.float64, torch.float32])
def test_feature_pnp_multi_matches_reference(tag, storage):
    """feature_pnp_multi (optimize_feature_pnp.py:20-47): three refine + find_inliers rounds.
    fp64 storage: the reference's pose to 1e-9 and its attributes; fp32 (f-only layout, fp64
    gradients in the LM kernel): pose within the north star's 1e-4 rad / 1e-4 m."""
    import json
    from collections import namedtuple
    z = load_npz("feature_pnp_multi")
    meta = json.loads(str(z["meta"]))
    Pred = namedtuple("Prediction", "points_3d reference_inliers matrix inlier_mask")
    pred = Pred(z["in_points_3d"], z["in_reference_inliers"], z["in_matrix"],
                z["in_mask_given"] if tag == "given" else None)
    q = torch.from_numpy(z["in_query"]).to(DEV)[None]
    r = torch.from_numpy(z["in_ref"]).to(DEV)[None]
    model = fmpnp.sparseFeaturePnP(meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss, lambda_=meta["lambda0"],
                                   storage=storage)
    fmpnp.config.configure(find_inliers_threshold=meta["find_inliers_threshold"])
    try:
        R, t, model = fmpnp.feature_pnp_multi(q, r, pred, z["in_K"], tuple(meta["image_shape"]), model=model)
    finally:
        fmpnp.config.configure(find_inliers_threshold=None)
    if storage == torch.float64:
        np.testing.assert_allclose(R.numpy(), z[f"out_R_{tag}"], atol=1e-9)
        np.testing.assert_allclose(t.numpy(), z[f"out_t_{tag}"], atol=1e-9)
        assert model.initial_cost_.item() == pytest.approx(float(z[f"initial_cost_{tag}"]), rel=1e-10)
        assert model.best_cost_.item() == pytest.approx(float(z[f"best_cost_{tag}"]), rel=1e-9)
        assert model.best_num_inliers_ == int(z[f"best_num_inliers_{tag}"])
    else:
        assert rot_angle(R.numpy(), z[f"out_R_{tag}"]) < 1e-4
        assert np.linalg.norm(t.numpy() - z[f"out_t_{tag}"]) < 1e-4


@pytest.mark.parametrize("wgs", [1, 3])
def test_async_launch_writes_every_result_field(wgs):
    """With one workgroup per problem the launch zeroes nothing (fmpnp_refine_batch_async):
    the kernel itself writes every field of every result, texel_gathers included.  The
    result buffer is filled with 0xFF bytes (NaN doubles, -1 integers) before each launch;
    the results must equal the synchronous refine's, with G = 1 and with a team (G = 3)."""
    inputs = synth.problem_inputs(300, 64, 60, 80, seed=78, device=DEV)
    feats = rf.pack_features(inputs["fmap"], storage=torch.float32, device=DEV)
    prob = rf.make_problem(feats, inputs["fref"], inputs["pts3d"], inputs["K"], inputs["im_width"],
                           inputs["im_height"], inputs["R0"], inputs["t0"])
    opts = rf.make_options(15, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=wgs)
    want = rf.refine([prob], opts)[0][0]
    ab = rf.AsyncBatch([prob] * 4, opts)
    for _ in range(2):
        ab.d_res.fill_(255)
        ab.launch()
        assert _lib.last_launch()["wgs_per_problem"] == wgs
        for r in ab.results():
            for k, v in want.items():
                assert np.array_equal(np.asarray(r[k]), np.asarray(v), equal_nan=True), k
