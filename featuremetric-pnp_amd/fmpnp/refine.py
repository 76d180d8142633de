"""Host-side plumbing of the HIP refiner: feature packing, problem descriptors,
synchronous and asynchronous batched refinement.

Everything here moves pointers and sizes into the C ABI of libfmpnp.so
(include/fmpnp.h); torch provides device memory and streams only.
"""
import ctypes
import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

_TORCH2CODE = {torch.float32: _lib.F32, torch.float64: _lib.F64}
_CODE2TORCH = {v: k for k, v in _TORCH2CODE.items()}


def _dtype_code(dt):
    if dt not in _TORCH2CODE:
        raise TypeError(f"feature dtype must be float32 or float64, got {dt}")
    return _TORCH2CODE[dt]


def _round4(c):
    return (c + 3) // 4 * 4


@dataclass
class PackedFeatures:
    """Channels-last feature texels on the device: buf[H][W][3][cstride] = (f, gx, gy)
    (layout "fgrad"), or buf[H][W][cstride] = f only (layout "f": the LM kernel forms the
    Sobel gradients with `sobel_flags` when it gathers a texel)."""
    buf: torch.Tensor
    C: int
    H: int
    W: int
    cstride: int
    layout: str = "fgrad"
    sobel_flags: int = 0

    @property
    def dtype(self):
        return self.buf.dtype

    @property
    def dtype_code(self):
        return _dtype_code(self.buf.dtype)


def _as_device(x, device, dtype=None, non_blocking=False):
    """Host or device array -> contiguous device tensor.  non_blocking: host data goes
    through pinned memory and an asynchronous copy on the current stream (the host does
    not wait for the device; torch's pinned allocator keeps the staging buffer alive
    until the copy ran)."""
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
    dt = dtype if dtype is not None else t.dtype
    if non_blocking and not t.is_cuda:
        return t.to(dtype=dt).contiguous().pin_memory().to(device=device, non_blocking=True)
    t = t.to(device=device, dtype=dt)
    return t.contiguous()


def pack_features(fmap, gx=None, gy=None, storage=None, device=None, sobel_normalized=False,
                  sobel_replicate_pad=False, stream=None, out=None, layout="fgrad"):
    """[C,H,W] (or [1,C,H,W]) feature map -> PackedFeatures.

    layout="f": the channels-last f plane only (a third of the bytes); the Sobel flags are
    recorded for the LM kernel, which computes the gradients itself (fp32 storage only).

    out: optional caller-owned contiguous device tensor [H, W, 3, cstride] ([H, W, cstride]
    for layout "f") of the storage dtype to pack into (cstride = C rounded up to 4; a padded
    one is zeroed first).

    Without gx/gy the Sobel gradients are computed on the device (fused kernel;
    vendored kornia Sobel by default: unnormalised, zero padded,
    featurePnP/helpers/sobel_pytorch.py).  With gx/gy they are packed as given
    (sparseFeaturePnP.forward receives them from its caller).
    """
    fmap = fmap if isinstance(fmap, torch.Tensor) else torch.as_tensor(np.asarray(fmap))
    if fmap.dim() == 4:
        fmap = fmap[0]
    if fmap.dim() != 3:
        raise ValueError("feature map must be [C,H,W] or [1,C,H,W]")
    device = torch.device(device) if device is not None else (
        fmap.device if fmap.is_cuda else torch.device("cuda", torch.cuda.current_device()))
    _lib.require_device(device)
    in_dt = fmap.dtype if fmap.dtype in _TORCH2CODE else torch.float32
    storage = storage or in_dt
    C, H, W = fmap.shape
    cs = _round4(C)
    if layout not in ("fgrad", "f"):
        raise ValueError("layout must be 'fgrad' or 'f'")
    if layout == "f" and (gx is not None or storage != torch.float32):
        raise ValueError("layout 'f' packs fp32 f only (the gradients are formed by the LM kernel)")
    oshape = (H, W, 3, cs) if layout == "fgrad" else (H, W, cs)
    with torch.cuda.device(device):
        f = _as_device(fmap, device, in_dt)
        gxd = gyd = None
        if gx is not None:
            gxd = _as_device(gx.reshape(C, H, W) if isinstance(gx, torch.Tensor) else np.asarray(gx).reshape(C, H, W),
                             device, in_dt)
            gyd = _as_device(gy.reshape(C, H, W) if isinstance(gy, torch.Tensor) else np.asarray(gy).reshape(C, H, W),
                             device, in_dt)
        if out is not None:
            if (tuple(out.shape) != oshape or out.dtype != storage or out.device != device
                    or not out.is_contiguous()):
                raise ValueError(f"out must be a contiguous {storage} tensor {list(oshape)} on {device}")
            if cs != C:
                out.zero_()
        elif cs != C:
            out = torch.zeros(oshape, dtype=storage, device=device)
        else:
            out = torch.empty(oshape, dtype=storage, device=device)
        s = stream if stream is not None else _lib.stream_ptr(device)
        if layout == "f":
            rc = _lib.load().fmpnp_pack_features_f(ctypes.c_void_p(f.data_ptr()), _dtype_code(in_dt), C, H, W,
                                                   ctypes.c_void_p(out.data_ptr()), _dtype_code(storage), cs, s)
        else:
            rc = _lib.load().fmpnp_pack_features(
                ctypes.c_void_p(f.data_ptr()), ctypes.c_void_p(gxd.data_ptr()) if gxd is not None else None,
                ctypes.c_void_p(gyd.data_ptr()) if gyd is not None else None, _dtype_code(in_dt), C, H, W,
                ctypes.c_void_p(out.data_ptr()), _dtype_code(storage), cs, int(bool(sobel_normalized)),
                int(bool(sobel_replicate_pad)), s)
        _lib.check(rc, "fmpnp_pack_features")
        # keep inputs alive until the kernel has consumed them
        if f.data_ptr() != fmap.data_ptr() or gxd is not None:
            torch.cuda.current_stream(device).synchronize()
    flags = int(bool(sobel_normalized)) | (int(bool(sobel_replicate_pad)) << 1)
    return PackedFeatures(out, C, H, W, cs, layout, flags if layout == "f" else 0)


def pad_reference(fref, cstride, storage, device):
    """fref [N,C] -> device [N, cstride] of the storage dtype (zero padded)."""
    fref = fref if isinstance(fref, torch.Tensor) else torch.as_tensor(np.asarray(fref))
    N, C = fref.shape
    out = torch.zeros((N, cstride), dtype=storage, device=device)
    out[:, :C] = fref.to(device=device, dtype=storage)
    return out


def gather_reference(ref_hc, reference_inliers, image_shape, cstride=None, storage=torch.float32, device=None,
                     err_flag=None):
    """Device fref gather of optimize_feature_pnp.py:51-56 -> [N, cstride].

    err_flag (a device int32 tensor of one element, zeroed by the caller): asynchronous
    form -- nothing waits for the device, an out-of-map inlier sets the flag (checked by
    the caller later) instead of raising here."""
    if ref_hc.dim() == 4:
        ref_hc = ref_hc[0]
    C, Hr, Wr = ref_hc.shape
    device = torch.device(device) if device is not None else (
        ref_hc.device if ref_hc.is_cuda else torch.device("cuda", torch.cuda.current_device()))
    _lib.require_device(device)
    in_dt = ref_hc.dtype if ref_hc.dtype in _TORCH2CODE else torch.float32
    cs = cstride or _round4(C)
    with torch.cuda.device(device):
        ref = _as_device(ref_hc, device, in_dt)
        if isinstance(reference_inliers, torch.Tensor) and reference_inliers.is_cuda:
            inl = reference_inliers.to(device=device, dtype=torch.float64).reshape(-1, 2).contiguous()
        else:
            inl = _as_device(torch.as_tensor(np.asarray(reference_inliers, dtype=np.float64).reshape(-1, 2)), device,
                             torch.float64, non_blocking=err_flag is not None)
        N = inl.shape[0]
        out = torch.zeros((N, cs), dtype=storage, device=device)
        if err_flag is not None:
            if not (err_flag.is_cuda and err_flag.dtype == torch.int32):
                raise TypeError("err_flag must be a device int32 tensor")
            rc = _lib.load().fmpnp_gather_reference_async(
                ctypes.c_void_p(ref.data_ptr()), _dtype_code(in_dt), C, Hr, Wr, ctypes.c_void_p(inl.data_ptr()), N,
                int(image_shape[0]), int(image_shape[1]), ctypes.c_void_p(out.data_ptr()), _dtype_code(storage), cs,
                ctypes.c_void_p(err_flag.data_ptr()), _lib.stream_ptr(device))
            _lib.check(rc, "fmpnp_gather_reference_async")
            return out
        rc = _lib.load().fmpnp_gather_reference(
            ctypes.c_void_p(ref.data_ptr()), _dtype_code(in_dt), C, Hr, Wr, ctypes.c_void_p(inl.data_ptr()), N,
            int(image_shape[0]), int(image_shape[1]), ctypes.c_void_p(out.data_ptr()), _dtype_code(storage), cs,
            _lib.stream_ptr(device))
        if rc == -1:
            raise IndexError("a reference inlier maps outside the reference hypercolumn "
                             "(optimize_feature_pnp.py:56 raises IndexError)")
        _lib.check(rc, "fmpnp_gather_reference")
    return out


def _mat(x, shape):
    a = np.asarray(x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else x, dtype=np.float64)
    return a.reshape(shape)


@dataclass
class Problem:
    """One refinement problem: packed query features + reference descriptors + points + pose."""
    feats: PackedFeatures
    fref: torch.Tensor          # device [N, ld] of feats.dtype
    pts3d: torch.Tensor         # device [N, 3] float64
    K: np.ndarray
    im_width: int
    im_height: int
    R0: np.ndarray
    t0: np.ndarray
    c_begin: int = 0
    c_end: int = None

    def descriptor(self):
        p = _lib.Problem()
        f = self.feats
        if self.fref.dtype != f.dtype:
            raise TypeError("fref and packed features must share a dtype")
        p.feat = f.buf.data_ptr()
        p.fref = self.fref.data_ptr()
        p.pts3d = self.pts3d.data_ptr()
        p.Hf, p.Wf, p.cstride = f.H, f.W, f.cstride
        p.c_begin = int(self.c_begin)
        p.c_end = int(f.C if self.c_end is None else min(self.c_end, f.C))
        p.ld_ref = self.fref.shape[1]
        p.N = self.pts3d.shape[0]
        p.im_width, p.im_height = int(self.im_width), int(self.im_height)
        p.K[:] = list(_mat(self.K, 9))
        p.R0[:] = list(_mat(self.R0, 9))
        p.t0[:] = list(_mat(self.t0, 3))
        return p


def make_problem(feats, fref, pts3d, K, im_width, im_height, R0, t0, c_begin=0, c_end=None, non_blocking=False):
    dev = feats.buf.device
    pts = _as_device(torch.as_tensor(np.asarray(pts3d.detach().cpu() if isinstance(pts3d, torch.Tensor) else pts3d,
                                                dtype=np.float64)).reshape(-1, 3), dev, torch.float64,
                     non_blocking) \
        if not (isinstance(pts3d, torch.Tensor) and pts3d.is_cuda and pts3d.dtype == torch.float64) \
        else pts3d.reshape(-1, 3).contiguous()
    if not (isinstance(fref, torch.Tensor) and fref.is_cuda and fref.dtype == feats.dtype
            and fref.shape[1] % 4 == 0):
        fref = pad_reference(fref, _round4(max(fref.shape[1], 1)), feats.dtype, dev)
    return Problem(feats, fref.contiguous(), pts, K, im_width, im_height, R0, t0, c_begin, c_end)


_SAMPLING = {"nearest": _lib.NEAREST, "bilinear": _lib.BILINEAR}


def bind_layout(problems, options):
    """The options with `layout` / `sobel_flags` taken from the problems' packed features
    (every problem of a launch shares one layout)."""
    lays = {(p.feats.layout, p.feats.sobel_flags) for p in problems}
    if len(lays) > 1:
        raise ValueError("all problems of a launch must share one feature layout")
    o = _lib.Options.from_buffer_copy(options)
    if lays:
        lay, flags = lays.pop()
        o.layout = _lib.LAYOUT_F if lay == "f" else _lib.LAYOUT_FGRAD
        o.sobel_flags = flags
    return o


def make_options(n_iters, lambda0=0.01, loss=_lib.SQUARED, barron_alpha=0.0, ratio_threshold=None,
                 dtype=_lib.F32, mode=_lib.MODE_FORWARD, wgs_per_problem=0, max_teams=0, memoize=True,
                 sampling="nearest", speculate=True, helpers=0):
    """fmpnp_options.  sampling: "nearest" (the reference's indexing_, model.py:74-97) or
    "bilinear" (extension: 2x2 taps of f, gx, gy; definition in fmpnp_device.h bilinear_taps,
    checked against the oracle's restatement -- no reference counterpart, parity unpinned).
    memoize: re-gather a point's texel only when it changed; speculate (memoised nearest
    forward runs): gather the predicted next texels beside the LM tail; helpers: first-evaluation
    helper workgroups per problem (0 = planner, < 0 = none, > 0 = cap).  None of them changes
    the results."""
    o = _lib.Options()
    o.mode = int(mode)
    o.n_iters = int(n_iters)
    o.lambda0 = float(lambda0)
    o.use_ratio = 0 if ratio_threshold is None else 1
    o.ratio_threshold = 0.0 if ratio_threshold is None else float(ratio_threshold)
    o.loss = int(loss)
    o.barron_alpha = float(barron_alpha)
    o.sampling = _SAMPLING[sampling] if isinstance(sampling, str) else int(sampling)
    o.dtype = int(dtype)
    o.wgs_per_problem = int(wgs_per_problem)
    o.max_teams = int(max_teams)
    o.no_memo = (0 if speculate else 2) if memoize else 1
    o.helpers = int(helpers)
    return o


def _result_dict(r):
    return dict(R=np.array(r.R[:]).reshape(3, 3), t=np.array(r.t[:]), initial_cost=r.initial_cost,
                best_cost=r.best_cost, final_lambda=r.final_lambda, final_lr=r.final_lr,
                best_num_inliers=r.best_num_inliers, n_evals=r.n_evals, n_steps=r.n_steps,
                n_accepted=r.n_accepted, status=r.status, has_best=bool(r.has_best),
                texel_gathers=int(r.texel_gathers))


def _trace_dict(entries, n):
    n = min(n, len(entries))
    return dict(R=np.array([entries[i].R[:] for i in range(n)]).reshape(-1, 3, 3),
                t=np.array([entries[i].t[:] for i in range(n)]).reshape(-1, 3),
                cost=np.array([entries[i].cost for i in range(n)]),
                lam=np.array([entries[i].lambda_after for i in range(n)]),
                lr=np.array([entries[i].lr_after for i in range(n)]),
                n_supported=np.array([entries[i].n_supported for i in range(n)]),
                n_kept=np.array([entries[i].n_kept for i in range(n)]),
                accepted=np.array([entries[i].accepted for i in range(n)], dtype=bool))


def refine(problems, options, trace=False):
    """Synchronous batched refinement.  Returns ([result dict], [trace dict] | None)."""
    n = len(problems)
    if n == 0:
        return [], ([] if trace else None)
    dev = problems[0].feats.buf.device
    _lib.require_device(dev)
    descs = (_lib.Problem * n)(*[p.descriptor() for p in problems])
    if descs[0].feat and options.dtype != problems[0].feats.dtype_code:
        raise TypeError("options.dtype does not match the packed features")
    options = bind_layout(problems, options)
    res = (_lib.Result * n)()
    stride = max(1, options.n_iters + 1) if trace else 0
    tr = (_lib.TraceEntry * (n * stride))() if trace else None
    with torch.cuda.device(dev):
        rc = _lib.load().fmpnp_refine_batch(descs, n, ctypes.byref(options), res, tr, stride, _lib.stream_ptr(dev))
    _lib.check(rc, "fmpnp_refine_batch")
    results = [_result_dict(r) for r in res]
    traces = None
    if trace:
        traces = [_trace_dict(tr[i * stride:(i + 1) * stride], results[i]["n_evals"]) for i in range(n)]
    for r in results:
        if r["status"] & _lib.STATUS_SYNC_TIMEOUT:
            raise _lib.FmpnpError("cross-workgroup exchange timed out (device oversubscribed?)")
    return results, traces


PROBLEM_DTYPE = np.dtype(_lib.Problem)   # fmpnp_problem as a numpy structured dtype (same layout)
RESULT_DTYPE = np.dtype(_lib.Result)


def results_from_array(arr):
    """fmpnp_result records (RESULT_DTYPE array) -> result dicts (as refine() returns)."""
    R, t = arr["R"].reshape(-1, 3, 3), arr["t"]
    cols = {k: arr[k].tolist() for k in ("initial_cost", "best_cost", "final_lambda", "final_lr", "best_num_inliers",
                                          "n_evals", "n_steps", "n_accepted", "status", "has_best", "texel_gathers")}
    return [dict(R=R[i].copy(), t=t[i].copy(), initial_cost=cols["initial_cost"][i], best_cost=cols["best_cost"][i],
                 final_lambda=cols["final_lambda"][i], final_lr=cols["final_lr"][i],
                 best_num_inliers=cols["best_num_inliers"][i], n_evals=cols["n_evals"][i],
                 n_steps=cols["n_steps"][i], n_accepted=cols["n_accepted"][i], status=cols["status"][i],
                 has_best=bool(cols["has_best"][i]), texel_gathers=int(cols["texel_gathers"][i]))
            for i in range(len(arr))]


class AsyncBatch:
    """Device-resident descriptors/results/workspace for repeated asynchronous launches
    (the bench's timed region: nothing but the LM kernel, plus two memsets when G > 1).

    Built from Problem objects, or (`from_descriptors`) from an fmpnp_problem array the
    caller filled column-wise -- the streamed pipeline's path, no per-query objects."""

    def __init__(self, problems, options, non_blocking=False):
        self.problems = list(problems)
        desc = np.zeros(len(self.problems), dtype=PROBLEM_DTYPE)
        for i, p in enumerate(self.problems):
            d = p.descriptor()
            desc[i] = np.frombuffer(ctypes.string_at(ctypes.addressof(d), PROBLEM_DTYPE.itemsize), PROBLEM_DTYPE)[0]
        self._setup(desc, bind_layout(self.problems, options), self.problems[0].feats.buf.device, non_blocking)

    @classmethod
    def from_descriptors(cls, desc, options, device, non_blocking=False):
        self = cls.__new__(cls)
        self.problems = []
        self._setup(desc, options, torch.device(device), non_blocking)
        return self

    def _setup(self, desc, options, dev, non_blocking):
        self.options = options
        self.n = n = len(desc)
        self.dev = dev
        _lib.require_device(self.dev)
        self.descs_np = np.ascontiguousarray(desc)
        self.descs_host = self.descs_np.ctypes.data_as(ctypes.POINTER(_lib.Problem))
        host = torch.from_numpy(self.descs_np.view(np.uint8))
        self.d_descs = torch.empty(host.numel(), dtype=torch.uint8, device=self.dev)
        self.d_descs.copy_(host.pin_memory() if non_blocking else host, non_blocking=non_blocking)
        self.d_res = torch.zeros(RESULT_DTYPE.itemsize * n, dtype=torch.uint8, device=self.dev)
        ws = _lib.load().fmpnp_workspace_size(self.descs_host, n, ctypes.byref(self.options))
        if ws == 0:
            raise _lib.FmpnpError("fmpnp_workspace_size failed (invalid problems/options)")
        self.d_ws = torch.empty(ws, dtype=torch.uint8, device=self.dev)
        self.ws_bytes = ws
        self.max_n = int(self.descs_np["N"].max()) if n else 0

    def launch(self, stream=None):
        s = stream if stream is not None else _lib.stream_ptr(self.dev)
        rc = _lib.load().fmpnp_refine_batch_async(
            ctypes.c_void_p(self.d_descs.data_ptr()), self.descs_host, self.n, self.max_n, ctypes.byref(self.options),
            ctypes.c_void_p(self.d_res.data_ptr()), None, 0, ctypes.c_void_p(self.d_ws.data_ptr()),
            self.ws_bytes, s)
        _lib.check(rc, "fmpnp_refine_batch_async")

    def results(self):
        torch.cuda.current_stream(self.dev).synchronize()
        return results_from_array(self.d_res.cpu().numpy().view(RESULT_DTYPE))


def point_costs(problem, R=None, t=None):
    """Per-point 0.5 ||f(p_i) - fref_i||^2 and support at (R, t) (default: the problem's
    R0, t0) on the device -- the projection, points_within_image and indexing_ of
    find_inliers (featurePnP/model.py:132-146), fmpnp_point_costs.  Returns device tensors
    (cost [N] fp64, 0 where unsupported; supported [N] bool)."""
    p = problem.descriptor()
    if R is not None:
        p.R0[:] = list(_mat(R, 9))
    if t is not None:
        p.t0[:] = list(_mat(t, 3))
    dev = problem.feats.buf.device
    N = int(p.N)
    cost = torch.zeros(N, dtype=torch.float64, device=dev)
    sup = torch.zeros(N, dtype=torch.int32, device=dev)
    lay = _lib.LAYOUT_F if problem.feats.layout == "f" else _lib.LAYOUT_FGRAD
    with torch.cuda.device(dev):
        rc = _lib.load().fmpnp_point_costs(ctypes.byref(p), lay, problem.feats.dtype_code,
                                           ctypes.c_void_p(cost.data_ptr()), ctypes.c_void_p(sup.data_ptr()),
                                           _lib.stream_ptr(dev))
    _lib.check(rc, "fmpnp_point_costs")
    return cost, sup.bool()


def compute_cost(problem, use_ratio=False, ratio_threshold=0.0):
    """compute_cost (featurePnP/model.py:216-243) at the problem's (R0, t0) on the device:
    fmpnp_compute_cost_async (per-point costs, one fixed-order reduction).  Returns the result
    dict (initial_cost; status NO_SUPPORT when no point is supported)."""
    p = problem.descriptor()
    dev = problem.feats.buf.device
    N = int(p.N)
    cost = torch.empty(max(N, 1), dtype=torch.float64, device=dev)
    sup = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
    res = torch.empty(RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    lay = _lib.LAYOUT_F if problem.feats.layout == "f" else _lib.LAYOUT_FGRAD
    with torch.cuda.device(dev):
        rc = _lib.load().fmpnp_compute_cost_async(ctypes.byref(p), lay, problem.feats.dtype_code, int(bool(use_ratio)),
                                                  float(ratio_threshold or 0.0), ctypes.c_void_p(cost.data_ptr()),
                                                  ctypes.c_void_p(sup.data_ptr()), ctypes.c_void_p(res.data_ptr()),
                                                  _lib.stream_ptr(dev))
    _lib.check(rc, "fmpnp_compute_cost_async")
    return results_from_array(res.cpu().numpy().view(RESULT_DTYPE))[0]


def project_pixels(R, t, pts3d, K):
    """Host restatement of the pixel projection (model.py:303-308) for track_['points2d'];
    elementwise numpy (no FMA), matching the device's sequential fp64 arithmetic."""
    R = np.asarray(R, dtype=np.float64)
    t = np.asarray(t, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64)
    X = np.asarray(pts3d, dtype=np.float64).reshape(-1, 3)
    P = [((R[i, 0] * X[:, 0] + R[i, 1] * X[:, 1]) + R[i, 2] * X[:, 2]) + t[i] for i in range(3)]
    u = [((K[i, 0] * P[0] + K[i, 1] * P[1]) + K[i, 2] * P[2]) for i in range(3)]
    with np.errstate(divide="ignore", invalid="ignore"):
        px = np.rint(u[0] / u[2]) - 1.0
        py = np.rint(u[1] / u[2]) - 1.0
    bad = ~np.isfinite(px) | ~np.isfinite(py) | (np.abs(px) > 2 ** 31 - 2) | (np.abs(py) > 2 ** 31 - 2)
    px = np.where(bad, -(2 ** 31), px)
    py = np.where(bad, -(2 ** 31), py)
    return np.stack([px, py], 1).astype(np.int32)


def nan_to_none(x):
    return None if (x is None or (isinstance(x, float) and math.isnan(x))) else x
