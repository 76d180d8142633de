"""The one-call façade path (fmpnp_feature_pnp: pack, gather, compute_cost and every level in one
host call with one host wait) against the step-by-step path (pack_features, gather_reference,
one refine per level) -- the same kernels on the same descriptors, so bit-identical poses,
attributes and track_ -- and against the reference's adapter goldens
(s2dhm/pose_prediction/optimize_feature_pnp.py:50-91)."""
import json
from collections import namedtuple

import numpy as np
import pytest
import torch

from golden_io import ADAPTER_CASES, load_npz

pytestmark = pytest.mark.gpu

import fmpnp  # noqa: E402
import importlib  # noqa: E402

from fmpnp import synth  # noqa: E402

ofp = importlib.import_module("fmpnp.optimize_feature_pnp")  # (the package re-exports the function under the module name)

DEV = "cuda:0"
Pred = namedtuple("Prediction", "points_3d reference_inliers matrix quaternion reference_filename")


def _run(one_call, monkeypatch, *args, **kw):
    if not one_call:
        monkeypatch.setattr(ofp, "_one_call_ok", lambda *a, **k: False)
    called = []
    real = ofp._feature_pnp_one_call

    def spy(*a, **k):
        called.append(1)
        return real(*a, **k)
    monkeypatch.setattr(ofp, "_feature_pnp_one_call", spy)
    try:
        R, t, m = fmpnp.feature_pnp(*args, **kw)
    finally:
        monkeypatch.undo()
    assert bool(called) == one_call
    return R, t, m


def _same(a, b):
    Ra, ta, ma = a
    Rb, tb, mb = b
    assert torch.equal(Ra, Rb) and torch.equal(ta, tb)
    for k in ("initial_cost_", "best_cost_"):
        va, vb = getattr(ma, k, None), getattr(mb, k, None)
        assert (va is None) == (vb is None), k
        if va is not None:
            assert torch.equal(va, vb), k
    assert getattr(ma, "best_num_inliers_", None) == getattr(mb, "best_num_inliers_", None)
    assert ma.status_ == mb.status_
    for k in ("Rs", "ts", "costs"):
        assert len(ma.track_[k]) == len(mb.track_[k]), k
        for x, y in zip(ma.track_[k], mb.track_[k]):
            assert (torch.equal(x, y) if isinstance(x, torch.Tensor) else x == y), k
    for x, y in zip(ma.track_["points2d"], mb.track_["points2d"]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("name", ADAPTER_CASES)
def test_one_call_equals_step_by_step_on_adapter_goldens(name, monkeypatch):
    z = load_npz(name)
    meta = json.loads(str(z["meta"]))
    pred = Pred(z["in_points_3d"], z["in_reference_inliers"], z["in_matrix"], np.array([1.0, 0, 0, 0]), "ref.png")
    q = torch.from_numpy(z["in_query"]).to(DEV)[None]
    r = torch.from_numpy(z["in_ref"]).to(DEV)[None]
    pyr = [tuple(lv) for lv in meta["pyramid"]] if meta["pyramid"] else None
    out = []
    for one in (True, False):
        model = fmpnp.sparseFeaturePnP(meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss, lambda_=meta["lambda0"],
                                       storage=torch.float64)
        out.append(_run(one, monkeypatch, q, r, pred, z["in_K"], tuple(meta["image_shape"]), track=True,
                        feature_pyramid=pyr, model=model))
    _same(*out)
    np.testing.assert_allclose(out[0][0].numpy(), z["out_R"], atol=1e-9)
    np.testing.assert_allclose(out[0][1].numpy(), z["out_t"], atol=1e-9)
    assert out[0][2].best_num_inliers_ == int(z["best_num_inliers_"])


def _synthetic(N, C, H, W, seed=11):
    (batch,), img = synth.pipeline_queries(1, 1, N, C, H, W, device=DEV, seed0=seed)
    q, r, p, K = batch[0]
    return q[None], r, Pred(p.points_3d, p.reference_inliers, p.matrix, np.array([1.0, 0, 0, 0]), "ref.png"), K, img


@pytest.mark.parametrize("shape,pyr", [((512, 256, 240, 320), None),
                                       ((295, 384, 64, 64), [(128, 384, None, None), (64, 128, None, None),
                                                              (0, 64, None, None)]),
                                       ((200, 96, 48, 64), [(32, 1000, None, None), (0, 32, None, None)])])
@pytest.mark.parametrize("storage", [torch.float32, torch.float64])
def test_one_call_equals_step_by_step_synthetic(shape, pyr, storage, monkeypatch):
    """cfg2 and channel pyramids (one level's end clamped by python slicing, model.py:194), fp32
    and fp64 storage, with track_ and the ratio test off."""
    q, r, pred, K, img = _synthetic(*shape)
    out = []
    for one in (True, False):
        model = fmpnp.sparseFeaturePnP(50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01, storage=storage)
        out.append(_run(one, monkeypatch, q, r, pred, K, img, track=True, feature_pyramid=pyr, model=model))
    _same(*out)


def test_one_call_ratio_without_track_and_layout_f(monkeypatch):
    """The ratio test (input_configs/full_robotcar_08.gin:40) without track_ takes the one-call path;
    the f-only layout too (fp32)."""
    q, r, pred, K, img = _synthetic(512, 256, 240, 320, seed=3)
    for kw in (dict(ratio_threshold=0.8), dict()):
        for layout in ("fgrad", "f"):
            out = []
            for one in (True, False):
                model = fmpnp.sparseFeaturePnP(50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                               storage=torch.float32, **kw)
                out.append(_run(one, monkeypatch, q, r, pred, K, img, model=model, layout=layout))
            _same(*out)


def test_one_call_raises_index_error_like_the_reference():
    """An inlier outside the reference map: optimize_feature_pnp.py:56 raises IndexError."""
    q, r, pred, K, img = _synthetic(64, 32, 40, 48, seed=5)
    inl = np.array(pred.reference_inliers, dtype=np.float64)
    inl[7] = (1e6, 5.0)
    bad = pred._replace(reference_inliers=inl)
    with pytest.raises(IndexError):
        fmpnp.feature_pnp(q, r, bad, K, img, model=fmpnp.sparseFeaturePnP(5))
    # the library stays usable after the error
    R, t, m = fmpnp.feature_pnp(q, r, pred, K, img, model=fmpnp.sparseFeaturePnP(5))
    assert m.status_ == 0


def test_one_call_no_support_returns_initial_pose_for_pyramids(monkeypatch):
    """multilevel_optimization with no supported point at the initial pose returns (R_init,
    t_init) and initial_cost_ None (model.py:183-187), as the step-by-step path."""
    q, r, pred, K, img = _synthetic(64, 32, 40, 48, seed=6)
    T = np.array(pred.matrix, dtype=np.float64)
    T[:3, 3] = (1e5, 0.0, 0.0)  # every point projects far outside the image
    away = pred._replace(matrix=T)
    pyr = [(16, 32, None, None), (0, 16, None, None)]
    out = []
    for one in (True, False):
        model = fmpnp.sparseFeaturePnP(10)
        out.append(_run(one, monkeypatch, q, r, away, K, img, feature_pyramid=pyr, model=model))
    assert out[0][2].initial_cost_ is None and out[1][2].initial_cost_ is None
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    np.testing.assert_array_equal(out[0][1].numpy(), T[:3, 3])


@pytest.mark.parametrize("shape,pyr,init", [((512, 256, 240, 320), None, "easy"),
                                            ((295, 384, 64, 64), [(128, 384, None, None), (0, 128, None, None)],
                                             "easy"),
                                            ((900, 192, 96, 96), [(64, 192, None, None), (0, 64, None, None)],
                                             "hard")])
def test_windowed_one_call_equals_full_pack(shape, pyr, init, monkeypatch):
    """fmpnp_feature_pnp with a packed window (only the texels near each point's initial texel are
    packed; a gather outside it re-runs the call fully packed) gives the full pack's results bit for
    bit -- at a radius that fits, and at radius 1 where points leave their windows (the re-run path);
    N = 900 (15 blocks) runs as a team of workgroups."""
    from fmpnp import _lib
    N, C, H, W = shape
    (batch,), img = synth.pipeline_queries(1, 1, N, C, H, W, device=DEV, seed0=21, init=init)
    q, r, p, K = batch[0]
    pred = Pred(p.points_3d, p.reference_inliers, p.matrix, np.array([1.0, 0, 0, 0]), "ref.png")

    def run(win):
        model = fmpnp.sparseFeaturePnP(50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01, storage=torch.float32)
        return _run(True, monkeypatch, q[None], r, pred, K, img, track=True, feature_pyramid=pyr, model=model,
                    window=win)
    full = run(0)
    L = _lib.load()
    for win in (6, 1):
        before = L.fmpnp_feature_pnp_reruns()
        _same(run(win), full)
        if win == 1 and N >= 512:
            assert L.fmpnp_feature_pnp_reruns() > before  # (the points of these starts move > 1 texel)
