"""Adapter: feature_pnp / optimize_feature_pnp (s2dhm/pose_prediction/optimize_feature_pnp.py:50-91)
and the DirectPoseModel call surface named by the build's north star.

The reference copies the GPU hypercolumn to host fp64, gathers the reference
descriptors with a per-point python loop, runs the Sobel on the CPU and then the
LM loop on the CPU (optimize_feature_pnp.py:51-69).  Here the query hypercolumn
stays on the device: one fused Sobel + channels-last pack kernel, one gather
kernel for the reference descriptors, one LM launch.
"""
import numpy as np
import torch

from . import config
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
    map is packed once (f-only layout for fp32 texels); every round reuses it and the
    device fref.  Returns (R, t, model) like feature_pnp."""
    model = _new_model(model)
    q = query_hypercolumns[0] if query_hypercolumns.dim() == 4 else query_hypercolumns
    dev = q.device if q.is_cuda else torch.device("cuda", torch.cuda.current_device())
    storage = storage or model.storage or (torch.float64 if q.dtype == torch.float64 else torch.float32)
    layout = "f" if storage == torch.float32 and getattr(model, "sampling", "nearest") == "nearest" else "fgrad"
    feats = _rf.pack_features(q, storage=storage, device=dev, layout=layout)               # :28,31
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
                feature_pyramid=None, model=None, storage=None, layout=None):
    """optimize_feature_pnp.py:50-71.  Returns (R, t, model) with R, t fp64 CPU tensors.

    layout: None picks the f-only layout (FMPNP_LAYOUT_F: the LM kernel forms the fp64 Sobel
    gradients, a third of the pack's bytes) for fp32 texels with nearest sampling and no
    pyramid, else the packed f/gx/gy planes ("fgrad")."""
    model = _new_model(model)
    q = query_hypercolumns[0] if query_hypercolumns.dim() == 4 else query_hypercolumns
    dev = q.device if q.is_cuda else torch.device("cuda", torch.cuda.current_device())
    storage = storage or model.storage or (torch.float64 if q.dtype == torch.float64 else torch.float32)
    if layout is None:
        layout = ("f" if storage == torch.float32 and feature_pyramid is None
                  and getattr(model, "sampling", "nearest") == "nearest" else "fgrad")
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


def optimize_feature_pnp(query_hypercolumns, net, prediction, K, image_shape=None, track=False, feature_pyramid=None,
                         features="s2dhm", model=None, verbose=False):
    """optimize_feature_pnp.py:73-91.  Returns (list t, list quaternion, model)."""
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
