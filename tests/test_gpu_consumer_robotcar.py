"""The consumer's production call at its real shape, against the oracle (verdict r05 item 2).

sparse_to_dense_predictor.py:242-247 calls optimize_feature_pnp -> feature_pnp
(s2dhm/pose_prediction/optimize_feature_pnp.py:50-71) once per query with the RobotCar
hypercolumn: C = 1664 channels at 256x256 for a 1024x1024 image, and a channel pyramid
(input_configs/default_robotcar.gin:75, robotcar_feature_pyramid.gin:61).  fmpnp.feature_pnp
takes the one-call path (fmpnp_feature_pnp) with its defaults: fp32 storage, the packed
f/gx/gy planes and, for C > 256, a packed window of radius 6 around each point's initial texel,
whose LM launches run the _W kernel variants (the window check compiled in).

Checked here, at N = 295 (the median query) and 866 (the largest num_final_matches of
results/results_s2dhm/robotcar/summary.csv), both pyramids, easy and hard starts:
  * against oracle.multilevel (oracle/, the C restatement of model.py:178-213 and :245-494 on the
    fp64 map and its fp64 Sobel, the reference's fref gather): per-evaluation support counts and
    evaluation counts identical on every level, costs within 1e-6 relative, final pose within
    1e-4 rad / 1e-4 m (north star), initial_cost_ / best_cost_ / best_num_inliers_;
  * the windowed call bit-identical to the same call fully packed (window=0), and no re-run;
  * the LM launches were the _W variants (fmpnp.last_launch())."""
import math
from collections import namedtuple

import numpy as np
import pytest
import torch

import oracle.oracle as orc

pytestmark = pytest.mark.gpu

import fmpnp  # noqa: E402
from fmpnp import _lib, synth  # noqa: E402

DEV = "cuda:0"
ITERS = 50
SEED = 23
Pred = namedtuple("Prediction", "points_3d reference_inliers matrix quaternion reference_filename")
PYRAMIDS = {"default_robotcar": [(640, 1664, None, None), (128, 640, None, None), (0, 128, None, None)],
            "robotcar_feature_pyramid": [(1024, 2048, None, None), (256, 1024, None, None), (0, 256, None, None)]}


def rot_angle(Ra, Rb):
    c = (np.trace(np.asarray(Ra).T @ np.asarray(Rb)) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


_MAPS = {}


def host_maps(q):
    """The query map (every case shares seed SEED's) in fp64 with its fp64 Sobel (the oracle's)."""
    if not _MAPS:
        fm = q[0].double().cpu().numpy()
        _MAPS["m"] = (fm,) + tuple(orc.sobel(fm))
    return _MAPS["m"]


def query(N, init):
    (batch,), img = synth.pipeline_queries(1, 1, N, 1664, 256, 256, device=DEV, seed0=SEED, init=init)
    q, r, p, K = batch[0]
    assert img == (1024, 1024)
    return q[None], r, Pred(p.points_3d, p.reference_inliers, p.matrix, np.array([1.0, 0, 0, 0]), "ref.png"), K, img


def call(args, pyr, window=None, track=True):
    model = fmpnp.sparseFeaturePnP(ITERS, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01)
    R, t, m = fmpnp.feature_pnp(*args, track=track, feature_pyramid=pyr, model=model, window=window)
    return R, t, m


@pytest.mark.parametrize("N", [295, 866])
@pytest.mark.parametrize("name", sorted(PYRAMIDS))
@pytest.mark.parametrize("init", ["easy", "hard"])
def test_consumer_call_at_robotcar_shape(N, name, init):
    pyr = PYRAMIDS[name]
    args = query(N, init)
    q, r, pred, K, img = args
    reruns = _lib.load().fmpnp_feature_pnp_reruns()
    R, t, m = call(args, pyr)
    what = f"N={N} {name} {init}"
    assert _lib.load().fmpnp_feature_pnp_reruns() == reruns, what  # (radius 6: no point left its window)
    assert _lib.last_launch()["variant_name"] in ("GM_W", "GM_H_W"), (what, _lib.last_launch())
    assert m.status_ == 0, what
    # the same call fully packed: bit-identical
    Rf, tf, mf = call(args, pyr, window=0)
    assert _lib.last_launch()["variant_name"] in ("GM", "GM_H", "GM_SPEC", "GM_SPEC_H"), what
    assert torch.equal(R, Rf) and torch.equal(t, tf), what
    assert torch.equal(m.best_cost_, mf.best_cost_) and m.best_num_inliers_ == mf.best_num_inliers_, what
    assert [float(c) for c in m.track_["costs"]] == [float(c) for c in mf.track_["costs"]], what
    # the oracle: the reference's preamble (fref gather, R, t from prediction.matrix) and multilevel
    fm, gx, gy = host_maps(q)
    fref = orc.gather_reference_features(fm, pred.reference_inliers, img)
    T = np.asarray(pred.matrix, dtype=np.float64)
    pts = np.asarray(pred.points_3d, dtype=np.float64).reshape(-1, 3)
    oR, ot, attrs, otr = orc.multilevel(pyr, pts, fref, fm, gx, gy, np.asarray(K, dtype=np.float64), img[0], img[1],
                                        T[:3, :3], T[:3, 3], ITERS, loss="geman_mcclure", trace_cap=ITERS + 1)
    ocost = np.concatenate([tr["cost"] for _, tr in otr])
    onsup = np.concatenate([tr["n_supported"] for _, tr in otr])
    nsup = np.array([int(mk.sum()) for mk in m.track_["mask"]])
    assert len(m.track_["costs"]) == len(ocost), what
    np.testing.assert_array_equal(nsup, onsup, err_msg=what)
    np.testing.assert_allclose(np.asarray(m.track_["costs"], dtype=np.float64), ocost, rtol=1e-6, err_msg=what)
    assert rot_angle(R.numpy(), oR) < 1e-4, what
    assert np.linalg.norm(t.numpy() - ot) < 1e-4, what
    assert float(m.initial_cost_) == pytest.approx(attrs["initial_cost"], rel=1e-6), what
    assert float(m.best_cost_) == pytest.approx(attrs["best_cost"], rel=1e-6), what
    assert m.best_num_inliers_ == attrs["best_num_inliers"], what
