"""DirectPoseModel().optimize_feature_pnp(...) -- the call surface BASELINE.json's north star
names -- driven the way the reference's predictor drives optimize_feature_pnp
(s2dhm/pose_prediction/sparse_to_dense_predictor.py:243-257; the stand-in for the broken
s2dhm/run_featurePnP.py:243), checked against the reference's own adapter outputs
(tests/golden/adapter_*.npz, produced by feature_pnp / optimize_feature_pnp themselves).
"""
import inspect
import json
from collections import namedtuple

import numpy as np
import pytest
import torch

import fmpnp
from golden_io import load_npz

Prediction = namedtuple("Prediction", "points_3d reference_inliers matrix quaternion reference_filename success "
                                      "num_matches")


def _case(name):
    z = load_npz(name)
    meta = json.loads(str(z["meta"]))
    pred = Prediction(z["in_points_3d"], z["in_reference_inliers"], z["in_matrix"], np.array([1.0, 0, 0, 0]),
                      "ref.png", True, len(z["in_points_3d"]))
    return z, meta, pred


def test_surface_signatures():
    """Same parameter names as the reference adapter (optimize_feature_pnp.py:50,73)."""
    dpm = fmpnp.DirectPoseModel()
    p = list(inspect.signature(dpm.optimize_feature_pnp).parameters)
    assert p[:7] == ["query_hypercolumns", "net", "prediction", "K", "image_shape", "track", "feature_pyramid"]
    p = list(inspect.signature(dpm.feature_pnp).parameters)
    assert p[:6] == ["query_hypercolumns", "reference_hypercolumns", "prediction", "K", "image_shape", "track"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["adapter_square", "adapter_pyramid"])
def test_direct_pose_model_like_the_predictor(name, capsys):
    z, meta, pred = _case(name)
    dev = "cuda:0"
    C, Hq, Wq = z["in_query"].shape
    # the predictor's hypercolumn is [1, C, H, W] on the GPU and goes in as .view(C, W, H)[None]
    query_dense_hypercolumn = torch.from_numpy(z["in_query"]).to(dev)[None]
    ref = torch.from_numpy(z["in_ref"]).to(dev)[None]

    class Net:  # ImageRetrievalModel.compute_hypercolumn (network.py:110-176): the reference map
        def compute_hypercolumn(self, names, to_cpu=False, resize=True):
            assert names == ["ref.png"] and not to_cpu
            return ref, None

    pyr = [tuple(l) for l in meta["pyramid"]] if meta["pyramid"] else None
    dpm = fmpnp.DirectPoseModel(n_iters=meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss, lambda_=meta["lambda0"],
                                storage=torch.float64)
    t, quaternion, model = dpm.optimize_feature_pnp(query_dense_hypercolumn.view(C, Wq, Hq)[None, ...], net=Net(),
                                                    prediction=pred, K=z["in_K"],
                                                    image_shape=tuple(meta["image_shape"]), track=True,
                                                    feature_pyramid=pyr)
    np.testing.assert_allclose(np.array(quaternion), z["opt_quat"], atol=1e-9)
    np.testing.assert_allclose(np.array(t), z["opt_t"], atol=1e-9)
    # the reference adapter's progress lines, printed unconditionally (optimize_feature_pnp.py:76,90)
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "Initial : {}".format(list(pred.quaternion) + list(pred.matrix[:3, 3]))
    assert out[-1] == "Final : {}".format(list(quaternion) + list(t))
    # the predictor's CSV row and export (sparse_to_dense_predictor.py:255-257)
    export = np.zeros(8)
    export[1:5], export[5:] = quaternion, t
    row = [pred.reference_filename, "query.png", pred.num_matches, model.best_num_inliers_,
           model.initial_cost_.item(), model.best_cost_.item(), None]
    assert row[3] == int(z["best_num_inliers_"])
    assert row[4] == pytest.approx(float(z["initial_cost_"]), rel=1e-10)
    assert row[5] == pytest.approx(float(z["best_cost_"]), rel=1e-9)
    if "track_costs" in z and pyr is None:
        np.testing.assert_allclose(np.array(model.track_["costs"]), z["track_costs"], rtol=1e-10)
    assert set(model.track_) == {"Rs", "ts", "costs", "points2d", "mask", "threshold_mask"}


@pytest.mark.gpu
def test_direct_pose_model_feature_pnp_fp32():
    """The default (fp32 hypercolumn) path: f-only layout, pose within the north star's 1e-4."""
    z, meta, pred = _case("adapter_nonsquare")
    dev = "cuda:0"
    dpm = fmpnp.DirectPoseModel(n_iters=meta["n_iters"], loss_fn="geman_mcclure_loss", lambda_=meta["lambda0"])
    R, t, model = dpm.feature_pnp(torch.from_numpy(z["in_query"]).float().to(dev)[None],
                                  torch.from_numpy(z["in_ref"]).float().to(dev)[None], pred, z["in_K"],
                                  tuple(meta["image_shape"]))
    c = (np.trace(R.numpy().T @ z["out_R"]) - 1) / 2
    assert np.arccos(min(1.0, c)) < 1e-4
    assert np.linalg.norm(t.numpy() - z["out_t"]) < 1e-4
