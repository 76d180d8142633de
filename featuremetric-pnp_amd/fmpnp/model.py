"""sparseFeaturePnP -- drop-in for featurePnP/model.py:155-494 running on the MI355X.

Same constructor, methods, arguments, return values and attributes as the
reference class; the LM loop itself is one HIP launch (libfmpnp.so).  Inputs may
be CPU or GPU tensors / numpy arrays; outputs are fp64 CPU tensors like the
reference's (model.py:491-494).

Feature storage precision: fp64 inputs are kept in fp64 on the device (results
match the reference to ~1e-15), fp32 inputs in fp32 (the reference's fp64 cast of
an fp32 hypercolumn is exact, so only the Sobel gradients are rounded).  Pass
`storage=torch.float32` to force fp32 texels for speed.
"""
import math
import warnings

import numpy as np
import torch
from torch import nn

from . import _lib
from . import config as _config
from . import losses as _losses
from . import refine as _rf


def _to_np(x, shape=None):
    a = x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
    a = a.astype(np.float64)
    return a.reshape(shape) if shape is not None else a


class sparseFeaturePnP(nn.Module):
    """featurePnP/model.py:155-168 (ctor), :170-176 (track), :178-213 (multilevel),
    :216-243 (compute_cost), :245-494 (forward)."""

    def __init__(self, n_iters, loss_fn=_losses.squared_loss, lambda_=0.01, verbose=False, ratio_threshold=None,
                 useGPU=False, storage=None, device=None, wgs_per_problem=0, sampling="nearest"):
        super().__init__()
        self.loss_fn = loss_fn  # (a module-valued loss keeps nn.Module's registration)
        # the plain attributes in one update (none is a tensor or a module: __setattr__ would
        # route each to object.__setattr__ anyway)
        self.__dict__.update(
            iterations=n_iters, verbose=verbose, lambda_=lambda_,
            track_={"Rs": [], "ts": [], "costs": [], "points2d": [], "mask": [], "threshold_mask": []},
            use_ratio_test_=ratio_threshold is not None, ratio_threshold_=ratio_threshold, initial_cost_=None,
            useGPU=useGPU,  # accepted for compatibility: the refiner always runs on the GPU
            storage=storage, device=device, wgs_per_problem=wgs_per_problem,
            sampling=sampling,  # extension: "bilinear" samples 2x2 taps (the reference: "nearest")
            status_=None, last_result_=None)

    def __setattr__(self, name, value):
        # plain attributes (iterations, loss_fn, the status and result fields) skip nn.Module's
        # parameter / buffer / submodule bookkeeping: a model is built per query by the consumer
        # (gin, optimize_feature_pnp.py:63), so its construction is part of every call's latency.
        # Tensors (initial_cost_, best_cost_) and modules keep nn.Module's path.
        if isinstance(value, (torch.Tensor, nn.Module)) or name in self.__dict__.get("_parameters", ()) \
                or name in self.__dict__.get("_buffers", ()) or name in self.__dict__.get("_modules", ()):
            nn.Module.__setattr__(self, name, value)
        else:
            object.__setattr__(self, name, value)

    # -- reference API --------------------------------------------------------
    def track(self, R, t, cost, points_2d, mask, threshold_mask):
        self.track_["Rs"].append(R)
        self.track_["ts"].append(t)
        self.track_["costs"].append(cost)
        self.track_["points2d"].append(points_2d)
        self.track_["mask"].append(mask)
        self.track_["threshold_mask"].append(threshold_mask)

    def _device(self, *tensors):
        if self.device is not None:
            return torch.device(self.device)
        for t in tensors:
            if isinstance(t, torch.Tensor) and t.is_cuda:
                return t.device
        return torch.device("cuda", torch.cuda.current_device())

    def _options(self, storage_code, mode=_lib.MODE_FORWARD, loss=None):
        code, alpha = _losses.resolve(self.loss_fn) if loss is None else (loss, 0.0)
        return _rf.make_options(self.iterations, self.lambda_, code, alpha,
                                self.ratio_threshold_ if self.use_ratio_test_ else None, storage_code, mode,
                                self.wgs_per_problem, sampling=self.sampling)

    def _storage_for(self, fmap):
        if self.storage is not None:
            return self.storage
        dt = fmap.dtype if isinstance(fmap, torch.Tensor) else torch.as_tensor(np.asarray(fmap)).dtype
        return torch.float64 if dt == torch.float64 else torch.float32

    def forward(self, pts3D, feature_ref, feature_map_query, feature_grad_x, feature_grad_y, K, im_width, im_height,
                R_init=None, t_init=None, track=False, confidence=None, scale=None):
        """model.py:245-494.  Returns (R_best, t_best) as fp64 CPU tensors."""
        dev = self._device(feature_map_query, pts3D)
        storage = self._storage_for(feature_map_query)
        feats = _rf.pack_features(feature_map_query, feature_grad_x, feature_grad_y, storage=storage, device=dev)
        return self._forward_packed(feats, pts3D, feature_ref, K, im_width, im_height, R_init, t_init, track)

    def _forward_packed(self, feats, pts3D, feature_ref, K, im_width, im_height, R_init=None, t_init=None,
                        track=False, c_begin=0, c_end=None):
        R0 = np.eye(3) if R_init is None else _to_np(R_init, (3, 3))          # model.py:271-273
        t0 = np.array([1.0, 1.0, 0.0]) if t_init is None else _to_np(t_init, (3,))  # model.py:275-276
        pts_np = _to_np(pts3D, (-1, 3))
        # a channel-sliced level uses columns [c_begin, c_end) of the full-width fref
        prob = _rf.make_problem(feats, feature_ref, pts3D if isinstance(pts3D, torch.Tensor) else pts_np, _to_np(K, (3, 3)),
                                im_width, im_height, R0, t0, c_begin, c_end)
        opts = self._options(feats.dtype_code)
        want_trace = bool(track) or bool(self.verbose)
        (res,), traces = _rf.refine([prob], opts, trace=want_trace)
        return self._apply_result(res, traces[0] if traces is not None else None, pts_np, K, im_width, im_height,
                                  track, prob)

    def _apply_result(self, res, tr, pts_np, K, im_width, im_height, track, prob=None):
        """One forward's result (and trace) -> the reference's attributes, track_ entries and
        verbose lines (model.py:347-361, 464-468, 477-494); returns (R, t) as fp64 CPU tensors."""
        self.last_result_ = res
        # (FMPNP_STATUS_HELPER_WAIT is informational -- a first-evaluation helper workgroup was not
        # resident in time and the main workgroup gathered itself, results unchanged -- so it is not
        # part of the model's status: status_ == 0 means success, as for the reference)
        self.status_ = res["status"] & ~_lib.STATUS_HELPER_WAIT
        if res["has_best"]:
            self.best_cost_ = torch.tensor(res["best_cost"], dtype=torch.float64)
            self.best_num_inliers_ = int(res["best_num_inliers"])
            if self.initial_cost_ is None:
                self.initial_cost_ = torch.tensor(res["initial_cost"], dtype=torch.float64)
        if tr is not None:
            Kn = _to_np(K, (3, 3))
            for k in range(len(tr["cost"])):
                if self.verbose:
                    print("Iter " if k == 0 else "new cost is ", tr["cost"][k])
                if track:
                    p2d = _rf.project_pixels(tr["R"][k], tr["t"][k], pts_np, Kn)
                    mask = (p2d[:, 0] >= 0) & (p2d[:, 1] >= 0) & (p2d[:, 0] < im_width) & (p2d[:, 1] < im_height)
                    self.track(torch.from_numpy(tr["R"][k].copy()), torch.from_numpy(tr["t"][k].copy()),
                               float(tr["cost"][k]), torch.from_numpy(p2d), torch.from_numpy(mask),
                               self._threshold_mask(prob, tr["R"][k], tr["t"][k]))
        if res["status"] & _lib.STATUS_NAN:
            warnings.warn("NaN detected, exit (model.py:411-413)")
        return (torch.from_numpy(res["R"].copy()), torch.from_numpy(res["t"].copy()))

    def _threshold_mask(self, prob, R, t):
        """track_["threshold_mask"] at (R, t) (model.py:328,452): the ratio test's mask over the
        supported points, from the device per-point costs; None without the ratio test."""
        if not self.use_ratio_test_:
            return None
        cost, sup = _rf.point_costs(prob, R, t)
        rho = torch.abs(self.loss_fn(cost[sup])[0])
        if rho.numel() == 0:
            return torch.zeros(0, dtype=torch.bool)
        return (rho < torch.max(rho) * self.ratio_threshold_).cpu()

    def compute_cost(self, pts3D, R, t, feature_map_query, feature_ref, K, im_width, im_height):
        """model.py:216-243: mean 0.5||e||^2 (no loss_fn, optional ratio test); None if no support."""
        dev = self._device(feature_map_query, pts3D)
        storage = self._storage_for(feature_map_query)
        fm = feature_map_query if isinstance(feature_map_query, torch.Tensor) else torch.as_tensor(
            np.asarray(feature_map_query))
        z = torch.zeros_like(fm)
        feats = _rf.pack_features(fm, z, z, storage=storage, device=dev)
        return self._compute_cost_packed(feats, pts3D, R, t, feature_ref, K, im_width, im_height)

    def _compute_cost_packed(self, feats, pts3D, R, t, feature_ref, K, im_width, im_height, c_begin=0, c_end=None):
        prob = _rf.make_problem(feats, feature_ref, pts3D, _to_np(K, (3, 3)), im_width, im_height, _to_np(R, (3, 3)),
                                _to_np(t, (3,)), c_begin, c_end)
        # one evaluation: per-point costs + one fixed-order reduction (fmpnp_compute_cost_async), the
        # same kernels as the one-call façade's multilevel path
        res = _rf.compute_cost(prob, self.use_ratio_test_, self.ratio_threshold_)
        if res["status"] & _lib.STATUS_NO_SUPPORT:
            return None
        return torch.tensor(res["initial_cost"], dtype=torch.float64)

    def multilevel_optimization(self, feature_pyramid, pts3D, feature_ref, feature_map_query, feature_grad_x,
                                feature_grad_y, *args, **kwargs):
        """model.py:178-213: coarse-to-fine over channel slices (optionally resized)."""
        K, im_width, im_height = args[0], args[1], args[2]
        R_init, t_init = kwargs.get("R_init"), kwargs.get("t_init")
        track = kwargs.get("track", False)
        dev = self._device(feature_map_query, pts3D)
        storage = self._storage_for(feature_map_query)
        fm = feature_map_query if isinstance(feature_map_query, torch.Tensor) else torch.as_tensor(
            np.asarray(feature_map_query))
        feats = _rf.pack_features(fm, feature_grad_x, feature_grad_y, storage=storage, device=dev)
        return self._multilevel_packed(feature_pyramid, feats, fm, pts3D, feature_ref, K, im_width, im_height,
                                       R_init, t_init, track)

    def _multilevel_packed(self, feature_pyramid, feats, fm, pts3D, feature_ref, K, im_width, im_height, R_init,
                           t_init, track):
        self.initial_cost_ = self._compute_cost_packed(feats, pts3D, R_init, t_init, feature_ref, K, im_width,
                                                       im_height)
        if self.initial_cost_ is None:  # model.py:183-187
            return R_init, t_init
        if feature_pyramid is None:
            return self._forward_packed(feats, pts3D, feature_ref, K, im_width, im_height, R_init, t_init, track)
        R, t = R_init, t_init
        C = feats.C
        fref_t = feature_ref if isinstance(feature_ref, torch.Tensor) else torch.as_tensor(np.asarray(feature_ref))
        for start, end, target_size, kernel_size in feature_pyramid:
            end_c = min(end, C)  # python slicing clamps (model.py:194)
            if target_size is None and kernel_size is None:
                R, t = self._forward_packed(feats, pts3D, fref_t, K, im_width, im_height, R, t, track,
                                            c_begin=start, c_end=end_c)
                continue
            # resized / blurred level (model.py:196-207): device resize and Gaussian in fp64 (the
            # reference's maps are fp64 here, optimize_feature_pnp.py:57), then the device Sobel + pack
            lvl = fm[start:end_c].to(feats.buf.device, dtype=torch.float64)[None]
            if target_size is not None:
                lvl = nn.functional.interpolate(lvl, size=(target_size, target_size), mode="bilinear")
            if kernel_size is not None:
                lvl = gaussian_blur(lvl, kernel_size, groups=end - start)
            lf = _rf.pack_features(lvl[0], storage=feats.dtype, device=feats.buf.device)
            R, t = self._forward_packed(lf, pts3D, fref_t[:, start:end_c], K, im_width, im_height, R, t, track)
        return R, t


def find_inliers(pts3D, R, t, feature_map_query, feature_ref, K, im_width, im_height, threshold=None, loss_fn=None,
                 mode=None, storage=None, device=None):
    """featurePnP/model.py:131-152 on the device: a bool mask [N] (CPU) of the points whose
    rounded projection at (R, t) lies in the image and whose loss of 0.5||f(p) - fref||^2
    passes the ratio test |rho| < max|rho| * threshold (ratio_threshold_feature_errors,
    model.py:120-129).  Projection, support and the per-point costs run in one HIP launch
    (fmpnp_point_costs); loss and ratio mask are N-element device tensor ops.

    threshold / loss_fn / mode default to the gin-style bindings of fmpnp.config
    (`configure(find_inliers_threshold=0.8)`; the reference's gin binds them).  Like the
    reference, a mode other than "ratio_max" returns None, a missing threshold raises
    TypeError, and an empty support set raises (torch.max of an empty tensor)."""
    fm = feature_map_query if isinstance(feature_map_query, torch.Tensor) else torch.as_tensor(
        np.asarray(feature_map_query))
    if fm.dim() == 4:
        fm = fm[0]
    if device is None:
        device = fm.device if fm.is_cuda else torch.device("cuda", torch.cuda.current_device())
    storage = storage or (torch.float64 if fm.dtype == torch.float64 else torch.float32)
    feats = _rf.pack_features(fm, storage=storage, device=device, layout="f" if storage == torch.float32 else "fgrad")
    return _find_inliers_packed(feats, pts3D, R, t, feature_ref, K, im_width, im_height, threshold, loss_fn, mode)


def _find_inliers_packed(feats, pts3D, R, t, feature_ref, K, im_width, im_height, threshold=None, loss_fn=None,
                         mode=None):
    cfg = _config.find_inliers_kwargs()
    threshold = cfg["threshold"] if threshold is None else threshold
    loss_fn = cfg["loss_fn"] if loss_fn is None else loss_fn
    mode = cfg["mode"] if mode is None else mode
    pts = pts3D if isinstance(pts3D, torch.Tensor) else np.asarray(pts3D, dtype=np.float64)
    prob = _rf.make_problem(feats, feature_ref, pts, _to_np(K, (3, 3)), im_width, im_height, _to_np(R, (3, 3)),
                            _to_np(t, (3,)))
    cost, sup = _rf.point_costs(prob)                                           # model.py:133-146
    if mode != "ratio_max":                                                     # model.py:149 (no else)
        return None
    if threshold is None:
        raise TypeError("find_inliers needs a threshold (the reference's gin binds find_inliers.threshold, "
                        "model.py:131; fmpnp.config.configure(find_inliers_threshold=...))")
    rho = loss_fn(cost[sup])[0]                                                 # model.py:147
    limit = torch.max(torch.abs(rho)) * threshold                               # model.py:122
    mask = sup.clone()
    mask[sup] = torch.abs(rho) < limit                                          # model.py:123,151
    return mask.cpu()


def gaussian_kernel2d(kernel_size, sigma=1.0):
    """kornia.filters.get_gaussian_kernel2d((k, k), (sigma, sigma)) as kornia 0.2.2 publishes it
    (requirements.txt:5): the 1-D window exp(-(i - k//2)^2 / (2 sigma^2)), i < k, in fp32,
    normalised by its fp32 sum, and the 2-D kernel as the fp32 outer product of the two
    windows.  An even or non-positive size raises TypeError, as kornia's
    get_gaussian_kernel1d does.  Parity unpinned: kornia is not importable here."""
    if not isinstance(kernel_size, int) or kernel_size <= 0 or kernel_size % 2 == 0:
        raise TypeError(f"kernel_size must be an odd positive integer. Got {kernel_size}")
    x = torch.arange(kernel_size, dtype=torch.float32) - kernel_size // 2
    g = torch.exp(-x.pow(2.0) / float(2 * sigma ** 2))
    g = g / g.sum()
    return torch.matmul(g.unsqueeze(-1), g.unsqueeze(-1).t())


def gaussian_blur(x, kernel_size, groups=None):
    """The blurred pyramid level of model.py:199-200: the fp32 kernel repeated `groups`
    (= end - start) times, as fp64, grouped conv2d with padding=1 (same size only for k=3;
    the reference keeps padding=1 for every k).  x: [1, C_level, H, W] fp64.  Like the
    reference, a level whose channel slice was clamped by Python slicing (end > C) has
    fewer channels than groups and raises RuntimeError."""
    groups = x.shape[1] if groups is None else int(groups)
    ker = gaussian_kernel2d(kernel_size)[None, None].repeat(groups, 1, 1, 1).to(device=x.device,
                                                                                 dtype=torch.float64)
    if x.shape[1] != groups:
        raise RuntimeError(f"Given groups={groups}, weight of size {list(ker.shape)}, expected input "
                           f"{list(x.shape)} to have {groups} channels, but got {x.shape[1]} channels instead "
                           "(model.py:199-200 with a pyramid level whose end exceeds the channel count)")
    return nn.functional.conv2d(x.to(torch.float64), ker, groups=groups, padding=1)


def is_nan(x):
    return x is None or (isinstance(x, float) and math.isnan(x))
