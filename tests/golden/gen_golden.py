#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the reference implementation.

TEST INFRASTRUCTURE ONLY.  This script imports the *reference* Python code
(aunagar/FeatureMetric-PnP, mounted read-only at /root/reference) and records
what it computes on small seeded inputs.  It refuses to run where the reference
is absent (e.g. on the GPU box); the committed .npz files are what travels.

How the reference is imported: featurePnP/model.py needs two
packages that are not installed in this image.  Stand-ins are written into a
temporary directory OUTSIDE the repository, ahead of the reference on sys.path:
  * gin    -- no-op `configurable` / `register` decorators (gin only binds
              defaults; every argument is passed explicitly below);
  * kornia -- `kornia.filters.spatial_gradient` routed to the reference's OWN
              vendored copy featurePnP/helpers/sobel_pytorch.SpatialGradient
              (unnormalised 3x3 Sobel, zero padding).  This is the Sobel that
              reproduces the notebook KAT bit-for-bit.
              kornia.filters.get_gaussian_kernel2d is NOT provided, so the
              pyramid's Gaussian-blur branch (model.py:198-200) is not pinned.
  * cv2    -- an empty module so that s2dhm/pose_prediction/matrix_utils.py
              (which uses cv2 only in matrix_from_se3) imports.

Every recorded quantity comes from the reference code itself:
  * per-iteration (g, H, lambda, lr, delta) by wrapping model.optimizer_step
    (model.py:37-72; forward calls it through the module global at :408);
  * the trial poses and costs from model.track_ (model.py:170-176,359,465);
  * best/initial cost and inlier count attributes (model.py:349-356,479-483).

Run:  python tests/golden/gen_golden.py      (writes tests/golden/*.npz)
"""
import json
import math
import os
import sys
import tempfile
from collections import namedtuple

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _install_shims():
    d = tempfile.mkdtemp(prefix="fmpnp_refshims_")
    os.makedirs(os.path.join(d, "kornia"))
    with open(os.path.join(d, "gin.py"), "w") as f:
        f.write(
            "def _deco(*a, **k):\n"
            "    if len(a) == 1 and callable(a[0]) and not k:\n"
            "        return a[0]\n"
            "    return lambda f: f\n"
            "configurable = _deco\n"
            "register = _deco\n")
    with open(os.path.join(d, "kornia", "__init__.py"), "w") as f:
        f.write("from . import filters\n")
    with open(os.path.join(d, "kornia", "filters.py"), "w") as f:
        f.write(
            "from helpers.sobel_pytorch import SpatialGradient\n"
            "def spatial_gradient(x):\n"
            "    return SpatialGradient()(x)\n")
    with open(os.path.join(d, "cv2.py"), "w") as f:
        f.write("# empty stand-in: matrix_utils uses cv2 only in matrix_from_se3\n")
    sys.path[:0] = [d, os.path.join(REF, "featurePnP"), os.path.join(REF, "s2dhm")]


if not os.path.isdir(os.path.join(REF, "featurePnP")):
    raise SystemExit("gen_golden.py needs the reference at /root/reference; "
                     "use the committed fixtures instead")
_install_shims()

import torch  # noqa: E402

torch.set_num_threads(1)
torch.set_default_dtype(torch.float32)

import model as refmodel  # noqa: E402  featurePnP/model.py
from helpers import utils as refutils  # noqa: E402  featurePnP/helpers/utils.py
from helpers.sobel_pytorch import SpatialGradient  # noqa: E402

# ----------------------------------------------------------------------------
# recorder around optimizer_step (model.py:37-72)
# ----------------------------------------------------------------------------
_REC = []
_orig_step = refmodel.optimizer_step


def _rec_step(g, H, lambda_=0, lr=1.0):
    delta = _orig_step(g, H, lambda_, lr=lr)
    _REC.append(dict(g=g.detach().clone().numpy(), H=H.detach().clone().numpy(),
                     lam=float(lambda_), lr=float(lr), delta=delta.detach().clone().numpy()))
    return delta


refmodel.optimizer_step = _rec_step

LOSSES = {
    "squared": refutils.squared_loss,
    "huber": refutils.huber_loss,
    "cauchy": refutils.cauchy_loss,
    "geman_mcclure": refutils.geman_mcclure_loss,
}


def loss_fn_for(name, alpha=None):
    if name == "barron":
        a = torch.tensor([float(alpha)]).double()
        return lambda x: refutils.barron_loss(x, a)
    return LOSSES[name]


def sobel_ref(fmap64):
    """featurePnP/helpers/utils.py:81-104 through the vendored kernel."""
    return refutils.sobel_filter(fmap64)


# ----------------------------------------------------------------------------
# seeded synthetic scenes (SURVEY.md §8d recipe, small sizes)
# ----------------------------------------------------------------------------
def make_fmap(rng, C, Hf, Wf):
    x = torch.from_numpy(rng.standard_normal((1, C, Hf, Wf)).astype(np.float32))
    x = torch.nn.functional.avg_pool2d(x, 7, stride=1, padding=3)
    x = x / x.norm(dim=1, keepdim=True).clamp_min(1e-12)
    return x[0].contiguous()  # [C,Hf,Wf] float32


def make_K(W, H, fscale=0.8, skew=0.0, fy_ratio=1.0):
    return np.array([[fscale * W, skew, W / 2.0],
                     [0.0, fscale * W * fy_ratio, H / 2.0],
                     [0.0, 0.0, 1.0]])


def make_points(rng, N, K, W, H, zlo=5.0, zhi=25.0):
    u = rng.uniform(0.1, 0.9, N) * W
    v = rng.uniform(0.1, 0.9, N) * H
    z = rng.uniform(zlo, zhi, N)
    fx, fy, cx, cy, s = K[0, 0], K[1, 1], K[0, 2], K[1, 2], K[0, 1]
    Y = (v - cy) * z / fy
    X = ((u - cx) - s * Y / z) * z / fx
    return np.stack([X, Y, z], 1)


def fref_identity(fmap64, pts, K, W, H):
    """feature_ref = reference NN gather (model.py:74-97) at the identity pose."""
    P = torch.from_numpy(pts)
    Kt = torch.from_numpy(K)
    p2d = torch.round(refutils.from_homogeneous(torch.mm(Kt, P.T).T)).type(torch.IntTensor) - 1
    m = refmodel.points_within_image(p2d, W, H)
    assert bool(m.all()), "identity projection must be inside the image"
    return refmodel.indexing_(fmap64, torch.flip(p2d, (1,)), W, H)


def rot_z(deg):
    a = math.radians(deg)
    return np.array([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]])


def rot_xyz(dx, dy, dz):
    def rx(a):
        a = math.radians(a)
        return np.array([[1, 0, 0], [0, math.cos(a), -math.sin(a)], [0, math.sin(a), math.cos(a)]])

    def ry(a):
        a = math.radians(a)
        return np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    return rot_z(dz) @ ry(dy) @ rx(dx)


# ----------------------------------------------------------------------------
# running the reference and packing its outputs
# ----------------------------------------------------------------------------
def _stack_track(model):
    tr = model.track_
    out = {}
    if tr["costs"]:
        out["track_costs"] = np.array(tr["costs"], dtype=np.float64)
        out["track_R"] = np.stack([r.numpy() for r in tr["Rs"]])
        out["track_t"] = np.stack([t.numpy() for t in tr["ts"]])
        out["track_npts"] = np.array([int(m.sum()) for m in tr["mask"]], dtype=np.int64)
        out["track_points2d"] = np.stack([p.numpy().astype(np.int64) for p in tr["points2d"]])
        out["track_mask"] = np.stack([m.numpy().astype(np.int8) for m in tr["mask"]])
    return out


def _rec_arrays():
    if not _REC:
        return {"rec_n": np.array(0)}
    return {
        "rec_n": np.array(len(_REC)),
        "rec_g": np.stack([r["g"] for r in _REC]),
        "rec_H": np.stack([r["H"] for r in _REC]),
        "rec_lam": np.array([r["lam"] for r in _REC]),
        "rec_lr": np.array([r["lr"] for r in _REC]),
        "rec_delta": np.stack([r["delta"] for r in _REC]),
    }


def _attrs(model):
    d = {}
    for k in ("best_cost_", "initial_cost_"):
        v = getattr(model, k, None)
        d[k] = np.array(np.nan if v is None else float(v))
        d["has_" + k] = np.array(v is not None)
    v = getattr(model, "best_num_inliers_", None)
    d["best_num_inliers_"] = np.array(-1 if v is None else int(v))
    return d


def run_forward(inp, opts):
    """sparseFeaturePnP.forward (model.py:245-494) or multilevel (model.py:178-213)."""
    _REC.clear()
    m = refmodel.sparseFeaturePnP(n_iters=opts["n_iters"],
                                  loss_fn=loss_fn_for(opts["loss"], opts.get("barron_alpha")),
                                  lambda_=opts["lambda0"], verbose=False,
                                  ratio_threshold=opts.get("ratio_threshold"), useGPU=False)
    pts = torch.from_numpy(inp["pts3d"])
    fref = torch.from_numpy(inp["fref"])
    fm = torch.from_numpy(inp["fmap"])
    gx = torch.from_numpy(inp["gx"])
    gy = torch.from_numpy(inp["gy"])
    K = torch.from_numpy(inp["K"])
    R0 = torch.from_numpy(inp["R0"])
    t0 = torch.from_numpy(inp["t0"])
    W, H = int(inp["im_width"]), int(inp["im_height"])
    if opts.get("pyramid") is not None:
        R, t = m.multilevel_optimization([tuple(l) for l in opts["pyramid"]], pts, fref, fm, gx, gy,
                                         K, W, H, R_init=R0, t_init=t0, track=True)
    else:
        R, t = m(pts, fref, fm, gx, gy, K, W, H, R_init=R0, t_init=t0, track=True)
    out = {"out_R": R.numpy().copy(), "out_t": t.numpy().copy()}
    out.update(_attrs(m))
    out.update(_stack_track(m))
    out.update(_rec_arrays())
    return out


def save_case(name, inp, opts, out, shared_fmap=None):
    arrs = {}
    for k, v in inp.items():
        if k == "fmap32" and shared_fmap is not None:
            continue
        arrs["in_" + k] = np.asarray(v)
    arrs.update(out)
    meta = dict(opts)
    if shared_fmap is not None:
        meta["shared_fmap"] = shared_fmap
    arrs["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print(f"{name}: evals={len(out.get('track_costs', []))} steps={int(out['rec_n'])} "
          f"best={float(out['best_cost_']):.6g} -> {path} ({os.path.getsize(path)} B)")


# ----------------------------------------------------------------------------
# cases
# ----------------------------------------------------------------------------
def case_kat_toy6():
    """Notebook KAT (FeatureBA_ToyExample.ipynb cells 14-28, toy 6)."""
    from PIL import Image
    d = os.path.join(REF, "featurePnP/toy_example/data")
    import pandas as pd
    df = pd.read_csv(os.path.join(d, "toyexample_6_data.csv"), sep=";", index_col=0)
    df = df[df["found"].astype(bool)]
    pts = df[["X", "Y", "Z"]].to_numpy(dtype=np.float64)
    p2d = df[["x", "y"]].to_numpy(dtype=np.float64)
    K = np.load(os.path.join(d, "toyexample_6_K.npy"))
    # cv2.imread(path, 0): R=G=B for this gray PNG, so the gray value is the red channel
    img = np.asarray(Image.open(os.path.join(d, "toyexample_6.png")))[..., 0].astype(np.float64)
    img_t = torch.from_numpy(img)[None]
    gx, gy = refutils.sobel_filter(img_t)
    coords = np.around(p2d).astype(int) - 1
    ref2d = torch.from_numpy(np.flip(coords, axis=1).copy())
    fref = torch.cat([img_t[:, i, j].unsqueeze(0) for i, j in zip(ref2d[:, 0], ref2d[:, 1])]).double()
    interp = torch.nn.functional.interpolate
    fm = interp(img_t.double().unsqueeze(0), size=(128, 128), mode="bilinear").squeeze(0)
    gx = interp(gx.unsqueeze(0), size=(128, 128), mode="bilinear").squeeze(0)
    gy = interp(gy.unsqueeze(0), size=(128, 128), mode="bilinear").squeeze(0)
    a = 4
    T = np.array([[math.cos(a * math.pi / 180), -math.sin(a * math.pi / 180), 0, 0],
                  [math.sin(a * math.pi / 180), math.cos(a * math.pi / 180), 0, 0],
                  [0, 0, 1, -0.1]])
    inp = dict(pts3d=pts, fref=fref.numpy(), fmap=fm.numpy(), gx=gx.numpy(), gy=gy.numpy(), K=K,
               R0=T[:, :3].copy(), t0=T[:, 3].copy(), im_width=img.shape[1], im_height=img.shape[0])
    opts = dict(n_iters=50, lambda0=0.01, loss="squared", ratio_threshold=None,
                kat_first=27497.41105769231, kat_last=276.125)
    out = run_forward(inp, opts)
    assert out["track_costs"][0] == 27497.41105769231 and out["track_costs"][-1] == 276.125, \
        (out["track_costs"][0], out["track_costs"][-1])
    save_case("kat_toy6", inp, opts, out)


def shared_scene(seed=0, C=16, Hf=48, Wf=64, N=128):
    rng = np.random.Generator(np.random.PCG64(seed))
    f32 = make_fmap(rng, C, Hf, Wf)
    W, H = 4 * Wf, 4 * Hf
    K = make_K(W, H)
    pts = make_points(rng, N, K, W, H)
    return rng, f32, K, pts, W, H


def base_inputs(f32, K, pts, W, H, R0, t0, fref=None):
    fm = f32.double()
    gx, gy = sobel_ref(fm)
    if fref is None:
        fref = fref_identity(fm, pts, K, W, H).numpy()
    return dict(pts3d=pts, fref=fref, fmap=fm.numpy(), gx=gx.numpy(), gy=gy.numpy(), K=K,
                R0=R0, t0=t0, im_width=W, im_height=H)


def strip_maps(inp):
    """The shared C=16 map travels once (fmap_c16.npz); cases keep only the small inputs."""
    return {k: v for k, v in inp.items() if k not in ("fmap", "gx", "gy")}


def main():
    case_kat_toy6()

    # --- shared C=16, 48x64 scene --------------------------------------------
    rng, f32, K, pts, W, H = shared_scene()
    fm = f32.double()
    gx, gy = sobel_ref(fm)
    np.savez_compressed(os.path.join(HERE, "fmap_c16.npz"), fmap32=f32.numpy(),
                        gx_sum=np.array(float(gx.sum())), gy_sum=np.array(float(gy.sum())),
                        gx_abs=np.array(float(gx.abs().sum())), gy_abs=np.array(float(gy.abs().sum())),
                        gx_probe=gx[:, ::7, ::9].numpy(), gy_probe=gy[:, ::7, ::9].numpy())
    R0 = rot_xyz(0.6, -0.4, 2.0)
    t0 = np.array([0.20, -0.12, 0.35])
    inp = base_inputs(f32, K, pts, W, H, R0, t0)
    cases = [
        ("gm_c16", dict(n_iters=30, lambda0=0.01, loss="geman_mcclure")),
        ("cauchy_c16", dict(n_iters=30, lambda0=0.01, loss="cauchy")),
        ("huber_c16", dict(n_iters=30, lambda0=0.01, loss="huber")),
        ("squared_c16", dict(n_iters=30, lambda0=0.01, loss="squared")),
        ("barron1_c16", dict(n_iters=25, lambda0=0.01, loss="barron", barron_alpha=1.0)),
        ("ratio08_gm", dict(n_iters=30, lambda0=0.01, loss="geman_mcclure", ratio_threshold=0.8)),
        ("ratio05_sq", dict(n_iters=20, lambda0=0.01, loss="squared", ratio_threshold=0.5)),
        ("lambda0_gm", dict(n_iters=20, lambda0=0.0, loss="geman_mcclure")),
        ("pyramid3_gm", dict(n_iters=15, lambda0=0.01, loss="geman_mcclure",
                             pyramid=[[8, 16, None, None], [4, 8, None, None], [0, 4, None, None]])),
        ("pyramid_clamp_sq", dict(n_iters=10, lambda0=0.01, loss="squared",
                                  pyramid=[[12, 40, None, None], [0, 12, None, None]])),
        ("pyramid_resize_sq", dict(n_iters=10, lambda0=0.01, loss="squared",
                                   pyramid=[[0, 8, 32, None], [8, 16, None, None]])),
        ("pyramid_ratio_gm", dict(n_iters=10, lambda0=0.01, loss="geman_mcclure", ratio_threshold=0.8,
                                  pyramid=[[4, 16, None, None], [0, 4, None, None]])),
    ]
    for name, opts in cases:
        opts.setdefault("ratio_threshold", None)
        out = run_forward(inp, opts)
        save_case(name, strip_maps(inp), opts, out, shared_fmap="fmap_c16")

    # points behind the camera (z<0 is not masked, model.py:113-117)
    pts_b = pts.copy()
    flip = rng.random(len(pts_b)) < 0.25
    pts_b[flip] *= -1.0
    inp_b = base_inputs(f32, K, pts_b, W, H, R0, t0)
    out = run_forward(inp_b, dict(n_iters=20, lambda0=0.01, loss="geman_mcclure", ratio_threshold=None))
    save_case("behind_camera_gm", strip_maps(inp_b), dict(n_iters=20, lambda0=0.01, loss="geman_mcclure",
                                                          ratio_threshold=None), out, shared_fmap="fmap_c16")

    # no support at the initial pose: early return of the current pose (model.py:316-320)
    inp_x = dict(inp)
    inp_x["t0"] = np.array([500.0, 0.0, 0.0])
    opts = dict(n_iters=10, lambda0=0.01, loss="squared", ratio_threshold=None)
    out = run_forward(inp_x, opts)
    save_case("no_support_init", strip_maps(inp_x), opts, out, shared_fmap="fmap_c16")

    # no support at a trial pose (model.py:441-445): a ramp map with a huge gradient
    # and tiny damping throws every point out of the image on the first step.
    rng2 = np.random.Generator(np.random.PCG64(7))
    C2, Hf2, Wf2 = 4, 24, 32
    yy, xx = np.meshgrid(np.arange(Hf2), np.arange(Wf2), indexing="ij")
    ramp = np.stack([xx * 3.0, yy * 2.0, (xx + yy) * 1.0, xx * yy * 0.1]).astype(np.float32)
    W2, H2 = 4 * Wf2, 4 * Hf2
    K2 = make_K(W2, H2)
    pts2 = make_points(rng2, 24, K2, W2, H2)
    f2 = torch.from_numpy(ramp)
    inp2 = base_inputs(f2, K2, pts2, W2, H2, rot_z(0.5), np.array([0.01, 0.0, 0.0]))
    inp2["fref"] = inp2["fref"] + 3000.0
    inp2["fmap32"] = ramp
    opts = dict(n_iters=10, lambda0=1e-6, loss="squared", ratio_threshold=None)
    out = run_forward(strip_fmap32(inp2), opts)
    save_case("no_support_trial", strip_maps(inp2), opts, out)

    # awkward geometry: C=5, non-integer stride, skewed K, fx != fy, non-square image
    rng3 = np.random.Generator(np.random.PCG64(3))
    C3, Hf3, Wf3 = 5, 37, 53
    f3 = make_fmap(rng3, C3, Hf3, Wf3)
    W3, H3 = 210, 150
    K3 = make_K(W3, H3, fscale=0.7, skew=0.5, fy_ratio=1.1)
    pts3 = make_points(rng3, 60, K3, W3, H3, 3.0, 12.0)
    inp3 = base_inputs(f3, K3, pts3, W3, H3, rot_xyz(1.0, 0.5, -1.5), np.array([-0.05, 0.04, 0.1]))
    inp3["fmap32"] = f3.numpy()
    for name, opts in [("odd_geom_gm", dict(n_iters=25, lambda0=0.01, loss="geman_mcclure")),
                       ("odd_geom_ratio_cauchy", dict(n_iters=25, lambda0=0.01, loss="cauchy",
                                                      ratio_threshold=0.6))]:
        opts.setdefault("ratio_threshold", None)
        out = run_forward(strip_fmap32(inp3), opts)
        save_case(name, strip_maps(inp3), opts, out)

    # compute_cost (model.py:216-243), with and without the ratio test
    cc = {}
    for thr in (None, 0.8):
        m = refmodel.sparseFeaturePnP(n_iters=1, ratio_threshold=thr)
        for tag, (R, t) in {"init": (R0, t0), "ident": (np.eye(3), np.zeros(3)),
                            "away": (np.eye(3), np.array([500.0, 0.0, 0.0]))}.items():
            v = m.compute_cost(torch.from_numpy(pts), torch.from_numpy(R), torch.from_numpy(t),
                               fm, torch.from_numpy(inp["fref"]), torch.from_numpy(K), W, H)
            cc[f"cost_{tag}_{thr}"] = np.array(np.nan if v is None else float(v))
    np.savez_compressed(os.path.join(HERE, "compute_cost.npz"), in_pts3d=pts, in_fref=inp["fref"],
                        in_K=K, in_R0=R0, in_t0=t0, in_im_width=W, in_im_height=H,
                        meta=np.array(json.dumps({"shared_fmap": "fmap_c16"})), **cc)

    # Sobel (helpers/utils.py:81-104 via sobel_pytorch.py) on a small map, fp64
    rng4 = np.random.Generator(np.random.PCG64(11))
    s = torch.from_numpy(rng4.standard_normal((3, 12, 17)))
    sgx, sgy = sobel_ref(s)
    np.savez_compressed(os.path.join(HERE, "sobel_small.npz"), x=s.numpy(), gx=sgx.numpy(), gy=sgy.numpy())

    # adapter: feature_pnp / optimize_feature_pnp (s2dhm/pose_prediction/optimize_feature_pnp.py)
    gen_adapter()


def strip_fmap32(inp):
    return {k: v for k, v in inp.items() if k != "fmap32"}


def gen_adapter():
    import functools
    import pose_prediction.optimize_feature_pnp as ofp
    from pose_prediction import matrix_utils
    Prediction = namedtuple("Prediction", "success num_matches num_inliers reference_inliers query_inliers "
                            "points_3d quaternion matrix reference_filename reference_keypoints inlier_mask")
    rng = np.random.Generator(np.random.PCG64(21))
    C, Hh, Wh = 8, 44, 44
    q32 = make_fmap(rng, C, Hh, Wh)
    r32 = make_fmap(rng, C, Hh, Wh)
    for case, image_shape, pyr in [("adapter_square", (192, 192), None),
                                   ("adapter_nonsquare", (200, 176), None),
                                   ("adapter_pyramid", (192, 192), [(4, 8, None, None), (0, 4, None, None)])]:
        Wimg, Himg = image_shape[0], image_shape[1]
        K = make_K(Wimg, Himg)
        N = 50
        pts = make_points(rng, N, K, Wimg, Himg)
        ref_inl = np.stack([rng.uniform(0, Wimg - 0.01, N), rng.uniform(0, Himg - 0.01, N)], 1)
        T = np.eye(4)
        T[:3, :3] = rot_xyz(0.5, -0.3, 1.5)
        T[:3, 3] = [0.1, -0.05, 0.2]
        pred = Prediction(True, N, N, ref_inl, None, pts.reshape(N, 1, 3), None, T, "ref.png", None, None)
        ofp.sparseFeaturePnP = functools.partial(refmodel.sparseFeaturePnP, n_iters=12,
                                                 loss_fn=refutils.geman_mcclure_loss, lambda_=0.01)
        _REC.clear()
        R, t, mdl = ofp.feature_pnp(q32[None], r32[None], pred, torch.from_numpy(K), image_shape,
                                    track=True, feature_pyramid=pyr)
        # optimize_feature_pnp (:73-91) with a stand-in network returning the reference map
        class _Net:
            def compute_hypercolumn(self, names, to_cpu=False, resize=True):
                return r32[None], None
        _REC.clear()
        tl, ql, mdl2 = ofp.optimize_feature_pnp(q32[None], _Net(), pred._replace(quaternion=np.array([1., 0, 0, 0])),
                                                K, image_shape, track=False, feature_pyramid=pyr)
        Tq = np.eye(4)
        Tq[:3, :3] = R.numpy()
        Tq[3, :3] = t.numpy()
        out = dict(out_R=R.numpy(), out_t=t.numpy(), opt_t=np.array(tl), opt_quat=np.array(ql),
                   quat_direct=matrix_utils.matrix_quaternion(Tq))
        out.update(_attrs(mdl))
        out.update(_stack_track(mdl))
        meta = dict(n_iters=12, lambda0=0.01, loss="geman_mcclure", ratio_threshold=None,
                    image_shape=list(image_shape), pyramid=[list(l) for l in pyr] if pyr else None)
        np.savez_compressed(os.path.join(HERE, case + ".npz"), in_query=q32.numpy(), in_ref=r32.numpy(),
                            in_points_3d=pts.reshape(N, 1, 3), in_reference_inliers=ref_inl, in_matrix=T,
                            in_K=K, meta=np.array(json.dumps(meta)), **out)
        print(f"{case}: best={float(out['best_cost_']):.6g} quat={out['opt_quat']}")
    # matrix_quaternion on assorted rotations (matrix_utils.py:29-74), incl. the trace<=M33 branch
    Ms, Qs = [], []
    for k in range(12):
        ax = rng.standard_normal(3)
        ang = [0.1, 1.0, 2.5, 3.1, 3.14159][k % 5]
        ax /= np.linalg.norm(ax)
        Kx = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        R = np.eye(3) + math.sin(ang) * Kx + (1 - math.cos(ang)) * Kx @ Kx
        M = np.eye(4)
        M[:3, :3] = R
        M[3, :3] = rng.standard_normal(3)
        Ms.append(M)
        Qs.append(matrix_utils.matrix_quaternion(M))
    np.savez_compressed(os.path.join(HERE, "quaternion.npz"), M=np.stack(Ms), q=np.stack(Qs))


def gen_find_inliers():
    """find_inliers (model.py:131-152) on the shared C=16 scene, and feature_pnp_multi
    (optimize_feature_pnp.py:20-47) on the adapter maps with and without initial inliers.
    find_inliers.threshold = 0.8 is input_configs/robotcar_inlier_GN.gin:42's binding."""
    import functools
    import pose_prediction.optimize_feature_pnp as ofp

    def find_inliers_ref(pts3D, R, t, feature_map_query, feature_ref, K, im_width, im_height, threshold=None,
                         loss_fn=refutils.squared_loss, mode="ratio_max"):
        # model.py:132-152 line for line, from the reference's own functions.  The reference
        # body itself raises under torch 2.10 at :151 (`mask_supported[mask_supported] = ...`
        # writes through its own index: "some elements ... refer to a single memory
        # location"); the index is cloned here, which is what older torch did implicitly.
        points_3d = torch.mm(R, pts3D.T).T + t
        points_2d = torch.round(refutils.from_homogeneous(torch.mm(K, points_3d.T).T)).type(torch.IntTensor) - 1
        mask_supported = refmodel.points_within_image(points_2d, im_width, im_height)
        points_2d_supported = points_2d[mask_supported, :]
        error = refmodel.indexing_(feature_map_query, torch.flip(points_2d_supported, (1,)), im_width,
                                   im_height) - feature_ref[mask_supported]
        cost = 0.5 * (error ** 2).sum(-1)
        cost_full, weights, _ = loss_fn(cost)
        if mode == "ratio_max":
            threshold_mask = refmodel.ratio_threshold_feature_errors(cost_full, threshold=threshold)
            mask_supported[mask_supported.clone()] = threshold_mask
            return mask_supported

    rng, f32, K, pts, W, H = shared_scene()
    fm = f32.double()
    R0 = rot_xyz(0.6, -0.4, 2.0)
    t0 = np.array([0.20, -0.12, 0.35])
    fref = fref_identity(fm, pts, K, W, H).numpy()
    poses = {"init": (R0, t0), "ident": (np.eye(3), np.zeros(3)), "shift": (np.eye(3), np.array([2.5, 0.0, 0.0]))}
    out = {}
    for tag, (R, t) in poses.items():
        for loss in ("squared", "geman_mcclure", "cauchy"):
            for thr in (0.8, 0.5):
                m = find_inliers_ref(torch.from_numpy(pts), torch.from_numpy(R), torch.from_numpy(t), fm,
                                     torch.from_numpy(fref), torch.from_numpy(K), W, H, threshold=thr,
                                     loss_fn=loss_fn_for(loss))
                out[f"mask_{tag}_{loss}_{thr}"] = m.numpy().astype(np.int8)
    np.savez_compressed(os.path.join(HERE, "find_inliers.npz"), in_pts3d=pts, in_fref=fref, in_K=K, in_im_width=W,
                        in_im_height=H, **{f"in_R_{k}": v[0] for k, v in poses.items()},
                        **{f"in_t_{k}": v[1] for k, v in poses.items()},
                        meta=np.array(json.dumps({"shared_fmap": "fmap_c16", "poses": list(poses)})), **out)
    print("find_inliers:", {k: int(v.sum()) for k, v in out.items() if "0.8" in k})

    # track_["threshold_mask"] (model.py:328,359,452,465) of the ratio-test cases: one mask over the
    # supported points per tracked evaluation, stored padded to N (-1 = not supported)
    inp = base_inputs(f32, K, pts, W, H, R0, t0)
    for name, opts in (("ratio08_gm", dict(n_iters=30, lambda0=0.01, loss="geman_mcclure", ratio_threshold=0.8)),
                       ("ratio05_sq", dict(n_iters=20, lambda0=0.01, loss="squared", ratio_threshold=0.5))):
        m = refmodel.sparseFeaturePnP(n_iters=opts["n_iters"], loss_fn=loss_fn_for(opts["loss"]),
                                      lambda_=opts["lambda0"], ratio_threshold=opts["ratio_threshold"])
        m(torch.from_numpy(inp["pts3d"]), torch.from_numpy(inp["fref"]), torch.from_numpy(inp["fmap"]),
          torch.from_numpy(inp["gx"]), torch.from_numpy(inp["gy"]), torch.from_numpy(K), W, H,
          R_init=torch.from_numpy(R0), t_init=torch.from_numpy(t0), track=True)
        tm = np.full((len(m.track_["mask"]), len(pts)), -1, dtype=np.int8)
        for k, (sup, thm) in enumerate(zip(m.track_["mask"], m.track_["threshold_mask"])):
            tm[k, sup.numpy()] = thm.numpy().astype(np.int8)
        np.savez_compressed(os.path.join(HERE, f"track_thr_{name}.npz"), threshold_mask=tm,
                            track_costs=np.array(m.track_["costs"], dtype=np.float64),
                            meta=np.array(json.dumps({"case": name})))
        print(f"track_thr_{name}: {tm.shape}, kept per eval {[(r == 1).sum() for r in tm[:4]]}")

    Prediction = namedtuple("Prediction", "success num_matches num_inliers reference_inliers query_inliers "
                            "points_3d quaternion matrix reference_filename reference_keypoints inlier_mask")
    rng = np.random.Generator(np.random.PCG64(31))
    C, Hh, Wh = 8, 44, 44
    q32 = make_fmap(rng, C, Hh, Wh)
    r32 = make_fmap(rng, C, Hh, Wh)
    image_shape = (192, 192)
    Kc = make_K(*image_shape)
    N = 60
    pts = make_points(rng, N, Kc, *image_shape)
    ref_inl = np.stack([rng.uniform(0, image_shape[0] - 0.01, N), rng.uniform(0, image_shape[1] - 0.01, N)], 1)
    T = np.eye(4)
    T[:3, :3] = rot_xyz(0.4, -0.2, 1.0)
    T[:3, 3] = [0.08, -0.04, 0.15]
    ofp.sparseFeaturePnP = functools.partial(refmodel.sparseFeaturePnP, n_iters=10,
                                             loss_fn=refutils.geman_mcclure_loss, lambda_=0.01)
    ofp.find_inliers = functools.partial(find_inliers_ref, threshold=0.8)
    res = {}
    for tag, inl in (("none", None), ("given", np.arange(0, N, 2))):
        pred = Prediction(True, N, N, ref_inl, None, pts.reshape(N, 1, 3), None, T, "ref.png", None, inl)
        R, t, mdl = ofp.feature_pnp_multi(q32[None], r32[None], pred, torch.from_numpy(Kc), image_shape)
        res[f"out_R_{tag}"] = R.numpy()
        res[f"out_t_{tag}"] = t.numpy()
        res[f"initial_cost_{tag}"] = np.array(float(mdl.initial_cost_))
        res[f"best_cost_{tag}"] = np.array(float(mdl.best_cost_))
        res[f"best_num_inliers_{tag}"] = np.array(int(mdl.best_num_inliers_))
        print(f"feature_pnp_multi/{tag}: best={float(mdl.best_cost_):.6g} inliers={int(mdl.best_num_inliers_)}")
    np.savez_compressed(os.path.join(HERE, "feature_pnp_multi.npz"), in_query=q32.numpy(), in_ref=r32.numpy(),
                        in_points_3d=pts.reshape(N, 1, 3), in_reference_inliers=ref_inl, in_matrix=T, in_K=Kc,
                        in_mask_given=np.arange(0, N, 2),
                        meta=np.array(json.dumps(dict(n_iters=10, lambda0=0.01, loss="geman_mcclure",
                                                      find_inliers_threshold=0.8, image_shape=list(image_shape)))),
                        **res)


if __name__ == "__main__":
    if sys.argv[1:] == ["find_inliers"]:  # only the find_inliers / feature_pnp_multi fixtures
        gen_find_inliers()
    else:
        main()
        gen_find_inliers()
