"""FMPNP_LAYOUT_F: the f plane alone in HBM, the Sobel gradients formed by the LM kernel
when it gathers a texel (needs an MI355X).

For fp32 hypercolumns the in-gather gradients are the reference's fp64 Sobel of the map
(helpers/utils.py:81-104) without the fp32 rounding the packed gradients carry, so this
path is held to the fp64-storage tolerances against the oracle: identical per-evaluation
support counts and costs to 1e-9 relative (the packed fp32 path: 1e-6), final pose within
1e-6 rad / 1e-6 m.
"""
import math

import numpy as np
import pytest
import torch

import oracle.oracle as orc

pytestmark = pytest.mark.gpu

import fmpnp  # noqa: E402,F401
from fmpnp import _lib, refine as rf, synth  # noqa: E402

DEV = "cuda:0"


def rot_angle(Ra, Rb):
    c = (np.trace(np.asarray(Ra).T @ np.asarray(Rb)) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


def sobel_np(x, normalized, replicate):
    """3x3 Sobel cross-correlation (helpers/sobel_pytorch.py:9-59), zero or edge padding."""
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1)), mode="edge" if replicate else "constant")
    a, b, c2 = xp[:, :-2, :-2], xp[:, :-2, 1:-1], xp[:, :-2, 2:]
    d, e = xp[:, 1:-1, :-2], xp[:, 1:-1, 2:]
    g, h, k = xp[:, 2:, :-2], xp[:, 2:, 1:-1], xp[:, 2:, 2:]
    gx = ((-a + c2) + (-2.0 * d + 2.0 * e)) + (-g + k)
    gy = ((-a - 2.0 * b) - c2) + ((g + 2.0 * h) + k)
    s = 0.125 if normalized else 1.0
    return gx * s, gy * s


def oracle_run(inp, n_iters, loss="geman_mcclure", normalized=False, replicate=False):
    fm = inp["fmap"].double().cpu().numpy()
    gx, gy = sobel_np(fm, normalized, replicate)
    p = orc.make_problem(inp["pts3d"], inp["fref"].double().cpu().numpy(), fm, gx, gy, inp["K"], inp["im_width"],
                         inp["im_height"], inp["R0"], inp["t0"])
    return orc.forward(p, orc.make_options(n_iters, 0.01, loss), trace_cap=n_iters + 1)


def gpu_run(inp, n_iters, loss=_lib.GEMAN_MCCLURE, layout="f", storage=torch.float32, wgs=0, **sobel):
    feats = rf.pack_features(inp["fmap"], storage=storage, device=DEV, layout=layout,
                             sobel_normalized=sobel.get("normalized", False),
                             sobel_replicate_pad=sobel.get("replicate", False))
    prob = rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                           inp["R0"], inp["t0"])
    (res,), (tr,) = rf.refine([prob], rf.make_options(n_iters, 0.01, loss, dtype=feats.dtype_code,
                                                      wgs_per_problem=wgs), trace=True)
    return res, tr


def check(res, tr, ores, otr, pose_tol=1e-6):
    np.testing.assert_array_equal(tr["n_supported"], otr["n_supported"])
    np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-9)
    assert rot_angle(res["R"], ores["R"]) < pose_tol
    assert np.linalg.norm(np.asarray(res["t"]) - ores["t"]) < pose_tol


@pytest.mark.parametrize("shape", [(37, 20, 28), (64, 33, 40), (256, 24, 32)])
def test_pack_f_is_a_channels_last_copy(shape):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(shape, generator=g)
    feats = rf.pack_features(x, storage=torch.float32, device=DEV, layout="f")
    C = shape[0]
    buf = feats.buf.cpu().numpy()
    assert buf.shape == (shape[1], shape[2], feats.cstride)
    np.testing.assert_array_equal(buf[:, :, :C].transpose(2, 0, 1), x.numpy())
    assert not buf[:, :, C:].any()


def test_cfg2_shape_against_oracle():
    """BASELINE config 2 shape (N=512, C=256, 240x320, GM), 8 iterations: one-round
    16-byte gathers of the 3x3 neighbourhood."""
    inp = synth.problem_inputs(512, 256, 240, 320, seed=3, device=DEV)
    ores, otr = oracle_run(inp, 8)
    res, tr = gpu_run(inp, 8)
    check(res, tr, ores, otr)


def test_cfg5_shape_against_oracle_multi_round_and_team():
    """N=2048, C=512, 480x640, Cauchy: two channel rounds per lane, G >= 2 workgroups."""
    inp = synth.problem_inputs(2048, 512, 480, 640, seed=5, device=DEV)
    ores, otr = oracle_run(inp, 5, loss="cauchy")
    res, tr = gpu_run(inp, 5, loss=_lib.CAUCHY)
    assert _lib.last_launch()["wgs_per_problem"] >= 2
    check(res, tr, ores, otr)


def border_problem(C, Hf, Wf, seed):
    """Points whose texels cover the whole map, the border rows / columns included."""
    rng = np.random.default_rng(seed)
    fmap = synth.feature_map(C, Hf, Wf, seed, DEV)
    W, H = 4 * Wf, 4 * Hf
    K = np.array([[0.8 * W, 0.0, W / 2.0], [0.0, 0.8 * W, H / 2.0], [0.0, 0.0, 1.0]])
    n = 96
    u = np.concatenate([rng.uniform(0.5, 4.0, 16), rng.uniform(W - 4.0, W - 0.5, 16), rng.uniform(0.5, W - 0.5, 64)])
    v = np.concatenate([rng.uniform(0.5, H - 0.5, 32), rng.uniform(0.5, 4.0, 32), rng.uniform(H - 4.0, H - 0.5, 32)])
    z = rng.uniform(5.0, 25.0, n)
    X = np.stack([(u - K[0, 2]) * z / K[0, 0], (v - K[1, 2]) * z / K[1, 1], z], 1)
    fref = synth.reference_descriptors(fmap, X, K, W, H)
    return dict(fmap=fmap, fref=fref, pts3d=X, K=K, im_width=W, im_height=H, R0=synth.rot_z(0.3),
                t0=np.array([0.01, -0.02, 0.03]))


@pytest.mark.parametrize("normalized,replicate", [(False, False), (True, False), (False, True), (True, True)])
def test_border_texels_and_sobel_flags(normalized, replicate):
    """Neighbourhoods cut by the map edge: zero padding (the vendored kornia Sobel) or
    replicate padding, unnormalised or /8 -- the flags the pack kernel would take."""
    inp = border_problem(24, 18, 26, seed=7)
    ores, otr = oracle_run(inp, 12, normalized=normalized, replicate=replicate)
    res, tr = gpu_run(inp, 12, normalized=normalized, replicate=replicate)
    check(res, tr, ores, otr)


def test_unaligned_channels_take_the_scalar_gather():
    """C = 6 (cstride 8, the last vector half empty) and a map whose rows are not 16-byte
    multiples: the per-channel path."""
    inp = synth.problem_inputs(128, 6, 30, 45, seed=9, device=DEV)
    ores, otr = oracle_run(inp, 10)
    res, tr = gpu_run(inp, 10)
    check(res, tr, ores, otr)


def test_layout_f_independent_of_workgroups_per_problem():
    inp = synth.problem_inputs(512, 64, 60, 80, seed=4, device=DEV)
    r1, t1 = gpu_run(inp, 15, wgs=1)
    r4, t4 = gpu_run(inp, 15, wgs=4)
    assert np.array_equal(r1["R"], r4["R"]) and np.array_equal(r1["t"], r4["t"])
    assert np.array_equal(t1["cost"], t4["cost"])


def test_layout_f_close_to_fp64_packed_gradients():
    """The same fp64 gradients stored (fp64 packed layout) or formed in the gather (layout f):
    same trajectory to the summation order."""
    inp = synth.problem_inputs(512, 256, 240, 320, seed=8, device=DEV)
    rf_, tf = gpu_run(inp, 10)
    rd, td = gpu_run(inp, 10, layout="fgrad", storage=torch.float64)
    np.testing.assert_array_equal(tf["n_supported"], td["n_supported"])
    np.testing.assert_allclose(tf["cost"], td["cost"], rtol=1e-9)
    assert rot_angle(rf_["R"], rd["R"]) < 1e-6


def test_mixed_layouts_in_one_launch_are_refused():
    inp = synth.problem_inputs(64, 8, 12, 16, seed=1, device=DEV)
    pf = rf.pack_features(inp["fmap"], storage=torch.float32, device=DEV, layout="f")
    pg = rf.pack_features(inp["fmap"], storage=torch.float32, device=DEV)
    probs = [rf.make_problem(p, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"], inp["R0"],
                             inp["t0"]) for p in (pf, pg)]
    with pytest.raises(ValueError):
        rf.refine(probs, rf.make_options(3, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32))


def test_facade_feature_pnp_fp32_takes_layout_f():
    """feature_pnp on an fp32 hypercolumn packs f only (the default for fp32, nearest, no
    pyramid) and lands where the fp64 packed-gradient path lands."""
    ((query,),), img = synth.pipeline_queries(1, 1, N=256, C=64, Hf=60, Wf=80, device=DEV, seed0=77)
    q, r, pred, K = query
    Kt = torch.from_numpy(np.asarray(K, np.float64))
    R32, t32, m32 = fmpnp.feature_pnp(q[None], r, pred, Kt, img)
    R64, t64, m64 = fmpnp.feature_pnp(q[None], r, pred, Kt, img, storage=torch.float64)
    assert rot_angle(R32.numpy(), R64.numpy()) < 1e-6
    assert np.linalg.norm(t32.numpy() - t64.numpy()) < 1e-6
    np.testing.assert_allclose(m32.best_cost_.item(), m64.best_cost_.item(), rtol=1e-9)
    assert m32.best_num_inliers_ == m64.best_num_inliers_
