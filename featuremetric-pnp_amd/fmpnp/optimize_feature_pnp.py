"""Adapter: feature_pnp / optimize_feature_pnp (s2dhm/pose_prediction/optimize_feature_pnp.py:50-91)
and the DirectPoseModel call surface named by the build's north star.

The reference copies the GPU hypercolumn to host fp64, gathers the reference
descriptors with a per-point python loop, runs the Sobel on the CPU and then the
LM loop on the CPU (optimize_feature_pnp.py:51-69).  Here the query hypercolumn
stays on the device: one fused Sobel + channels-last pack kernel, one gather
kernel for the reference descriptors, one LM launch.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib, config
from . import refine as _rf
from .matrix_utils import matrix_quaternion
from .model import _find_inliers_packed, sparseFeaturePnP


def _new_model(model):
    if model is not None:
        return model
    return sparseFeaturePnP(**config.model_kwargs())  # "Parameters from gin!" (optimize_feature_pnp.py:63)


def feature_pnp_multi(query_hypercolumns, reference_hypercolumns, prediction, K, image_shape, track=False,
                      model=None, storage=None, rounds=3):
    """optimize_feature_pnp.py:20-47: refine on the current inliers, re-select the inliers
    with find_inliers at the new pose, three times.  The initial inliers are
    prediction.inlier_mask, or find_inliers at the initial pose when it is None.  The query
    map is packed once (f, gx, gy planes); every round reuses it and the
    device fref.  Returns (R, t, model) like feature_pnp."""
    model = _new_model(model)
    q = query_hypercolumns[0] if query_hypercolumns.dim() == 4 else query_hypercolumns
    dev = q.device if q.is_cuda else torch.device("cuda", torch.cuda.current_device())
    storage = storage or model.storage or (torch.float64 if q.dtype == torch.float64 else torch.float32)
    # (three LM launches and four point-cost launches on one map: the packed f/gx/gy planes, as
    # feature_pnp -- the LM reads 16C bytes per gathered texel from them against 40C from "f")
    feats = _rf.pack_features(q, storage=storage, device=dev, layout="fgrad")              # :28,31
    fref = _rf.gather_reference(reference_hypercolumns, prediction.reference_inliers, image_shape,
                                cstride=feats.cstride, storage=storage, device=dev)          # :21-26
    pts3D = np.asarray(prediction.points_3d, dtype=np.float64).reshape(-1, 3)               # :22
    T = np.asarray(prediction.matrix, dtype=np.float64)
    R, t = torch.from_numpy(T[:3, :3].copy()), torch.from_numpy(T[:3, 3].copy())             # :30-31
    Kt = K if isinstance(K, torch.Tensor) else torch.from_numpy(np.asarray(K, dtype=np.float64))
    W, H = image_shape[0], image_shape[1]
    if prediction.inlier_mask is not None:                                                  # :35-39
        inliers = torch.zeros(pts3D.shape[0], dtype=torch.bool)
        inliers[torch.as_tensor(np.asarray(prediction.inlier_mask))] = True
    else:
        print("No initial inliers found.")
        inliers = _find_inliers_packed(feats, pts3D, R, t, fref, Kt, W, H)
    for _ in range(rounds):                                                                 # :43-46
        idx = inliers.numpy()
        R, t = model._forward_packed(feats, pts3D[idx], fref[inliers.to(dev)], Kt, W, H, R, t, track)
        inliers = _find_inliers_packed(feats, pts3D, R, t, fref, Kt, W, H)
    return R, t, model


def feature_pnp(query_hypercolumns, reference_hypercolumns, prediction, K, image_shape, track=False,
                feature_pyramid=None, model=None, storage=None, layout=None, window=None):
    """optimize_feature_pnp.py:50-71.  Returns (R, t, model) with R, t fp64 CPU tensors.

    layout: None (default) packs the f/gx/gy planes ("fgrad": the fused Sobel + channels-last
    pack); "f" packs f only (FMPNP_LAYOUT_F: a third of the pack's bytes, the LM kernel forms
    the fp64 Sobel gradients of every texel it gathers).  One query per call is LM-bound, and
    the LM reads 16C bytes per gathered texel from "fgrad" against 40C from "f": cfg2, one
    call, pack + LM 66 + 259 us against 33 + 559 us (rocprofv3, profiles/r05_facade_*).

    window: the one-call path packs only the texels within `window` texels of each point's texel
    at the initial pose (fmpnp_feature_pnp; a point that leaves its window re-runs the call fully
    packed, so results are the full pack's bit for bit); None = window_radius(C, H, W, N), 0 = off."""
    model = _new_model(model)
    q = query_hypercolumns[0] if query_hypercolumns.dim() == 4 else query_hypercolumns
    dev = q.device if q.is_cuda else torch.device("cuda", torch.cuda.current_device())
    storage = storage or model.storage or (torch.float64 if q.dtype == torch.float64 else torch.float32)
    if layout is None:
        layout = "fgrad"
    levels = _channel_levels(feature_pyramid, q.shape[0])
    if _one_call_ok(model, q, reference_hypercolumns, feature_pyramid, levels, track, storage, layout):
        return _feature_pnp_one_call(model, q, reference_hypercolumns, prediction, K, image_shape, track, levels,
                                     storage, layout, window)
    feats = _rf.pack_features(q, storage=storage, device=dev, layout=layout)               # :57, :61
    fref = _rf.gather_reference(reference_hypercolumns, prediction.reference_inliers, image_shape,
                                cstride=feats.cstride, storage=storage, device=dev)          # :51-56
    pts3D = np.asarray(prediction.points_3d, dtype=np.float64).reshape(-1, 3)               # :52
    T = np.asarray(prediction.matrix, dtype=np.float64)
    R, t = torch.from_numpy(T[:3, :3].copy()), torch.from_numpy(T[:3, 3].copy())             # :59-60
    Kt = K if isinstance(K, torch.Tensor) else torch.from_numpy(np.asarray(K, dtype=np.float64))
    if feature_pyramid is None:                                                             # :64-69
        R, t = model._forward_packed(feats, pts3D, fref, Kt, image_shape[0], image_shape[1], R, t, track)
    else:
        R, t = model._multilevel_packed(feature_pyramid, feats, q, pts3D, fref, Kt, image_shape[0], image_shape[1],
                                        R, t, track)
    return R, t, model


def _channel_levels(feature_pyramid, C):
    """multilevel_optimization's levels (model.py:193-194) as channel ranges [start, min(end, C))
    when every level is a plain channel slice (no resize, no blur); None otherwise."""
    if feature_pyramid is None:
        return None
    out = []
    for start, end, target_size, kernel_size in feature_pyramid:
        if target_size is not None or kernel_size is not None:
            return None
        out.append((int(start), min(int(end), C)))  # python slicing clamps (model.py:194)
    return out


def _one_call_ok(model, q, r, feature_pyramid, levels, track, storage, layout):
    """fmpnp_feature_pnp runs the whole call (pack, gather, compute_cost, every level) with one
    host wait when both maps are device tensors of the same device and channel count and the
    pyramid is channel slices only; track_ with the ratio test needs the packed map for its
    threshold masks (fmpnp_point_costs), so that case takes the step-by-step path."""
    r = r[0] if r.dim() == 4 else r
    ok = (q.is_cuda and r.is_cuda and q.device == r.device and q.dim() == 3 and r.dim() == 3
          and q.dtype in (torch.float32, torch.float64) and r.dtype in (torch.float32, torch.float64)
          and r.shape[0] == q.shape[0] and storage in (torch.float32, torch.float64)
          and not (track and model.use_ratio_test_) and (layout == "fgrad" or storage == torch.float32))
    if feature_pyramid is not None:
        ok = ok and levels is not None and len(levels) > 0 and all(0 <= a < b for a, b in levels)
    return ok


def window_radius(C, H, W, N):
    """The one-call path's default pack window (texels): FMPNP_FACADE_WINDOW overrides."""
    env = os.environ.get("FMPNP_FACADE_WINDOW")
    if env is not None:
        return int(env)
    # wide maps only: the windowed pack saves the writes of the unmarked texels (RobotCar C = 1664 at
    # 256x256, 295 / 866 points: 1.57 -> 1.42 / 1.97 -> 1.88 ms per call), but a window turns the
    # speculative gathers off (cfg2, C = 256: 0.450 -> 0.465 ms); radius 6: no re-run over the
    # synthetic starts at radii >= 5 (profiles/r05_facade_window_sweep.txt)
    return 6 if C > 256 else 0


_DP = ctypes.POINTER(ctypes.c_double)


def _feature_pnp_one_call(model, q, r, prediction, K, image_shape, track, levels, storage, layout, window=None):
    """feature_pnp through fmpnp_feature_pnp: one host call, one host wait (optimize_feature_pnp.py:50-71)."""
    r = r[0] if r.dim() == 4 else r
    q, r = q.contiguous(), r.contiguous()
    dev = q.device
    C, H, W = q.shape
    opts = model._options(_rf._dtype_code(storage))
    opts.layout = _lib.LAYOUT_F if layout == "f" else _lib.LAYOUT_FGRAD
    opts.sobel_flags = 0
    inl = np.ascontiguousarray(np.asarray(prediction.reference_inliers, dtype=np.float64).reshape(-1, 2))  # :53
    pts = np.ascontiguousarray(np.asarray(prediction.points_3d, dtype=np.float64).reshape(-1, 3))          # :52
    if inl.shape[0] != pts.shape[0]:
        raise ValueError("reference_inliers and points_3d must have one row per match")
    T = np.asarray(prediction.matrix, dtype=np.float64)
    R0, t0 = np.ascontiguousarray(T[:3, :3]), np.ascontiguousarray(T[:3, 3])                            # :59-60
    Kn = np.ascontiguousarray((K.detach().cpu().numpy() if isinstance(K, torch.Tensor) else np.asarray(K))
                              .astype(np.float64).reshape(3, 3))
    n_lv = len(levels) if levels else 0
    if window is None:
        window = window_radius(C, H, W, pts.shape[0])
    if layout != "fgrad" or getattr(model, "sampling", "nearest") != "nearest":
        window = 0
    lv = (_lib.Level * n_lv)(*[_lib.Level(a, b) for a, b in levels]) if n_lv else None
    res = np.zeros(n_lv + 1 if n_lv else 1, dtype=_rf.RESULT_DTYPE)
    want_trace = bool(track) or bool(model.verbose)
    stride = model.iterations + 1
    tr = (_lib.TraceEntry * (max(n_lv, 1) * stride))() if want_trace else None
    # (c_void_p arguments take plain addresses; the device switch only when the map is not on the current one)
    args = (q.data_ptr(), _rf._dtype_code(q.dtype), C, H, W, r.data_ptr(), _rf._dtype_code(r.dtype), r.shape[0],
            r.shape[1], r.shape[2], inl.ctypes.data, pts.ctypes.data, pts.shape[0], Kn.ctypes.data_as(_DP),
            R0.ctypes.data_as(_DP), t0.ctypes.data_as(_DP), int(image_shape[0]), int(image_shape[1]), lv, n_lv,
            ctypes.byref(opts), int(window), res.ctypes.data, tr, stride if want_trace else 0)
    if dev.index == torch.cuda.current_device():
        rc = _lib.load().fmpnp_feature_pnp(*args, _lib.stream_ptr(dev))
    else:
        with torch.cuda.device(dev):
            rc = _lib.load().fmpnp_feature_pnp(*args, _lib.stream_ptr(dev))
    if rc == _lib.ERANGE:
        raise IndexError("a reference inlier maps outside the reference hypercolumn "
                         "(optimize_feature_pnp.py:56 raises IndexError)")
    _lib.check(rc, "fmpnp_feature_pnp")
    out = _rf.results_from_array(res)
    if any(x["status"] & _lib.STATUS_SYNC_TIMEOUT for x in out):
        raise _lib.FmpnpError("cross-workgroup exchange timed out (device oversubscribed?)")
    W_img, H_img = image_shape[0], image_shape[1]

    def trace_of(i, n_evals):
        return _rf._trace_dict(tr[i * stride:(i + 1) * stride], n_evals) if want_trace else None
    if not n_lv:                                                                            # :64-65
        R, t = model._apply_result(out[0], trace_of(0, out[0]["n_evals"]), pts, Kn, W_img, H_img, track)
        return R, t, model
    # multilevel_optimization (model.py:178-213): initial_cost_ from compute_cost; no support -> the
    # initial pose, unrefined (:183-187); else each level's forward from the previous level's pose
    cost = out[0]
    if cost["status"] & _lib.STATUS_NO_SUPPORT:
        model.initial_cost_ = None
        return torch.from_numpy(R0.copy()), torch.from_numpy(t0.copy()), model
    model.initial_cost_ = torch.tensor(cost["initial_cost"], dtype=torch.float64)
    for li in range(n_lv):
        R, t = model._apply_result(out[1 + li], trace_of(li, out[1 + li]["n_evals"]), pts, Kn, W_img, H_img, track)
    return R, t, model


def optimize_feature_pnp(query_hypercolumns, net, prediction, K, image_shape=None, track=False, feature_pyramid=None,
                         features="s2dhm", model=None, verbose=True):
    """optimize_feature_pnp.py:73-91.  Returns (list t, list quaternion, model).  Prints the reference's
    "Initial : ..." / "Final : ..." lines (:76, :90) unless verbose=False (the reference always prints
    them; a consumer that scrapes stdout sees the same lines)."""
    cfg = config.adapter_kwargs()
    image_shape = image_shape if image_shape is not None else cfg.get("image_shape", (1024, 1024))
    if feature_pyramid is None:
        feature_pyramid = cfg.get("feature_pyramid")
    K = torch.from_numpy(np.asarray(K, dtype=np.float64))
    if verbose:
        print("Initial : {}".format(list(prediction.quaternion) + list(prediction.matrix[:3, 3])))
    if features == "d2-net":
        raise NotImplementedError("d2-net dense features are outside the refiner's scope")
    reference_hypercolumns, _ = net.compute_hypercolumn([prediction.reference_filename], to_cpu=False, resize=True)
    R, t, model = feature_pnp(query_hypercolumns, reference_hypercolumns, prediction, K, image_shape, track=track,
                              feature_pyramid=feature_pyramid, model=model)
    T = np.eye(4)
    T[:3, :3], T[3, :3] = R.numpy(), t.numpy()  # the reference writes t into the bottom row (:87)
    quaternion = matrix_quaternion(T)
    if verbose:
        print("Final : {}".format(list(quaternion) + list(t.numpy())))
    return list(t.numpy()), list(quaternion), model


class DirectPoseModel:
    """The call surface named by the build's north star: `.optimize_feature_pnp()` with the
    reference adapter's arguments, backed by the HIP refiner."""

    def __init__(self, **model_kwargs):
        self.model_kwargs = model_kwargs

    def make_model(self):
        kw = dict(config.model_kwargs())
        kw.update(self.model_kwargs)
        return sparseFeaturePnP(**kw)

    def feature_pnp_multi(self, query_hypercolumns, reference_hypercolumns, prediction, K, image_shape,
                          track=False):
        return feature_pnp_multi(query_hypercolumns, reference_hypercolumns, prediction, K, image_shape, track,
                                 model=self.make_model())

    def feature_pnp(self, query_hypercolumns, reference_hypercolumns, prediction, K, image_shape, track=False,
                    feature_pyramid=None):
        return feature_pnp(query_hypercolumns, reference_hypercolumns, prediction, K, image_shape, track,
                           feature_pyramid, model=self.make_model())

    def optimize_feature_pnp(self, query_hypercolumns, net, prediction, K, image_shape=None, track=False,
                             feature_pyramid=None, features="s2dhm"):
        return optimize_feature_pnp(query_hypercolumns, net, prediction, K, image_shape, track, feature_pyramid,
                                    features, model=self.make_model())
