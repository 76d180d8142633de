"""Coarse-to-fine refinement at the reference's production shapes, against the oracle.

1. The RobotCar hypercolumn (C = 128+256+256+512+512 = 1664 channels of hypercolumn_layers
   [9,14,17,21,24], network.gin:18; 256x256 map of a 1024x1024 image, image_shape of the
   robotcar input configs) with up to 866 points per query (the largest num_final_matches of
   results/results_s2dhm/robotcar/summary.csv), refined through sparseFeaturePnP.
   multilevel_optimization (featurePnP/model.py:178-213) with the two channel pyramids the
   reference's configs use:
     input_configs/default_robotcar.gin:75        [(640,1664), (128,640), (0,128)]
     input_configs/robotcar_feature_pyramid.gin:61 [(1024,2048), (256,1024), (0,256)]
   (the second one's first slice is clamped to [1024,1664) by Python slicing, model.py:194).
   The 1024-, 768-, 640- and 512-channel slices take the LM kernel's multi-round channel gathers
   (more than 64 V channels per half-wave lane), the full 1664 channels the compute_cost that
   sets initial_cost_ (model.py:182).
2. BASELINE.json configs[3] at its full shapes: C=512 @120x160 -> C=256 @240x320 -> C=128
   @480x640 (one map per level, the same points and 2560x1920 image, 50
   iterations per level, the pose chained from level to level as multilevel_optimization chains
   forward).

Both against the oracle (oracle/fmpnp_oracle.c; oracle.multilevel restates model.py:178-213):
identical per-evaluation support counts and evaluation counts on every level, costs within 1e-6
relative (fp32 texels and fp32-rounded packed gradients against the oracle's fp64 ones), final
pose within 1e-4 rad / 1e-4 m (BASELINE.json north star), and the model attributes.
"""
import math

import numpy as np
import pytest
import torch

import oracle.oracle as orc

pytestmark = pytest.mark.gpu

import fmpnp  # noqa: E402
from fmpnp import synth  # noqa: E402

DEV = "cuda:0"
ITERS = 50
PYRAMIDS = {"default_robotcar": [(640, 1664, None, None), (128, 640, None, None), (0, 128, None, None)],
            "robotcar_feature_pyramid": [(1024, 2048, None, None), (256, 1024, None, None), (0, 256, None, None)]}


def rot_angle(Ra, Rb):
    c = (np.trace(np.asarray(Ra).T @ np.asarray(Rb)) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


def _check_levels(track, otraces, what):
    ocost = np.concatenate([tr["cost"] for _, tr in otraces])
    onsup = np.concatenate([tr["n_supported"] for _, tr in otraces])
    nsup = np.array([int(m.sum()) for m in track["mask"]])
    assert len(track["costs"]) == len(ocost), what
    np.testing.assert_array_equal(nsup, onsup, err_msg=what)
    np.testing.assert_allclose(np.asarray(track["costs"]), ocost, rtol=1e-6, err_msg=what)


@pytest.mark.parametrize("name", sorted(PYRAMIDS))
@pytest.mark.parametrize("init", ["easy", "hard"])
def test_production_hypercolumn_pyramid(name, init):
    pyr = PYRAMIDS[name]
    inp = synth.problem_inputs(866, 1664, 256, 256, seed=17, device=DEV, init=init)
    assert (inp["im_width"], inp["im_height"]) == (1024, 1024)
    model = fmpnp.sparseFeaturePnP(ITERS, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01, storage=torch.float32)
    R, t = model.multilevel_optimization(pyr, inp["pts3d"], inp["fref"], inp["fmap"], None, None, inp["K"],
                                         inp["im_width"], inp["im_height"], R_init=inp["R0"], t_init=inp["t0"],
                                         track=True)
    fm = inp["fmap"].double().cpu().numpy()
    fref = inp["fref"].double().cpu().numpy()
    del inp["fmap"]
    gx, gy = orc.sobel(fm)
    oR, ot, attrs, otr = orc.multilevel(pyr, inp["pts3d"], fref, fm, gx, gy, inp["K"], inp["im_width"],
                                        inp["im_height"], inp["R0"], inp["t0"], ITERS, loss="geman_mcclure",
                                        trace_cap=ITERS + 1)
    what = f"{name} {init}"
    assert model.status_ == 0, what
    _check_levels(model.track_, otr, what)
    assert rot_angle(R.numpy(), oR) < 1e-4, what
    assert np.linalg.norm(t.numpy() - ot) < 1e-4, what
    assert float(model.initial_cost_) == pytest.approx(attrs["initial_cost"], rel=1e-6), what
    assert float(model.best_cost_) == pytest.approx(attrs["best_cost"], rel=1e-6), what
    assert model.best_num_inliers_ == attrs["best_num_inliers"], what


CONFIG3_LEVELS = [(512, 120, 160), (256, 240, 320), (128, 480, 640)]


def config3_level_inputs(level, seed, device=DEV):
    """configs[3] level `level` of query `seed`: that level's map (its own seed), the points and
    the 2560x1920 image of the finest level's scene, fref gathered from that level's map."""
    C, Hf, Wf = CONFIG3_LEVELS[level]
    X, K, W, H = synth.scene(512, 480, 640, seed)
    fmap = synth.feature_map(C, Hf, Wf, 10 * seed + level, device)
    fref = synth.reference_descriptors(fmap, X, K, W, H)
    return fmap, fref, X, K, W, H


@pytest.mark.parametrize("init", ["easy", "hard"])
def test_config3_pyramid_full_shapes(init):
    R0, t0 = synth.INITS[init]
    R, t = R0.copy(), t0.copy()
    oR, ot = R0.copy(), t0.copy()
    for level in range(3):
        fmap, fref, X, K, W, H = config3_level_inputs(level, seed=5)
        model = fmpnp.sparseFeaturePnP(ITERS, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01, storage=torch.float32)
        Rt, tt = model.forward(X, fref, fmap, None, None, K, W, H, R_init=R, t_init=t, track=True)
        fm = fmap.double().cpu().numpy()
        gx, gy = orc.sobel(fm)
        p = orc.make_problem(X, fref.double().cpu().numpy(), fm, gx, gy, K, W, H, oR, ot)
        ores, otr = orc.forward(p, orc.make_options(ITERS, 0.01, "geman_mcclure"), trace_cap=ITERS + 1)
        what = f"configs[3] level {level} {CONFIG3_LEVELS[level]} {init}"
        assert model.status_ == 0, what
        _check_levels(model.track_, [(ores, otr)], what)
        assert model.best_num_inliers_ == ores["best_num_inliers"], what
        R, t = Rt.numpy(), tt.numpy()
        oR, ot = ores["R"], ores["t"]
        assert rot_angle(R, oR) < 1e-4 and np.linalg.norm(t - ot) < 1e-4, what
