"""The CPU twin of the LM refiner (fmpnp_refine_batch_cpu, include/fmpnp.h).

An explicit CPU entry point over the same descriptors as fmpnp.refine.refine, with host
(numpy) buffers: the timed CPU baseline beside the GPU (bench.py's cpu_twin leg) and a parity
bridge for callers without a GPU.  Nothing in the GPU path calls it -- fmpnp.refine and the
façades raise without a gfx950 device instead of falling back here.

    feats = pack_host(fmap, gx, gy, np.float32)          # [Hf][Wf][3][cstride], fmpnp_pack_features' layout
    prob = problem_host(feats, fref, pts3d, K, W, H, R0, t0)
    results, traces = refine_cpu([prob], fmpnp.make_options(50, 0.01, _lib.GEMAN_MCCLURE), trace=True)
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .refine import _result_dict, _trace_dict


def _cs(c):
    return (int(c) + 3) // 4 * 4


def pack_host(fmap, gx=None, gy=None, dtype=np.float32, layout="fgrad"):
    """Channels-last host copy of [C, H, W] maps: [H][W][3][cstride] (f, gx, gy planes) or, with
    layout "f", [H][W][cstride] (f only; the twin forms the Sobel of a texel's 3x3 neighbourhood).
    Padding channels are zero."""
    fmap = np.asarray(fmap)
    C, H, W = fmap.shape
    cs = _cs(C)
    if layout == "f":
        out = np.zeros((H, W, cs), dtype=dtype)
        out[:, :, :C] = np.moveaxis(fmap, 0, -1)
        return out
    if gx is None or gy is None:
        raise ValueError("the fgrad layout takes the gradient maps (helpers/utils.py:81-104)")
    out = np.zeros((H, W, 3, cs), dtype=dtype)
    for k, m in enumerate((fmap, gx, gy)):
        out[:, :, k, :C] = np.moveaxis(np.asarray(m), 0, -1)
    return out


@dataclass
class HostProblem:
    feats: np.ndarray   # pack_host output
    layout: str
    C: int
    fref: np.ndarray    # [N, ld] of feats.dtype
    pts3d: np.ndarray   # [N, 3] float64
    K: np.ndarray
    im_width: int
    im_height: int
    R0: np.ndarray
    t0: np.ndarray
    c_begin: int = 0
    c_end: int = None

    def descriptor(self):
        p = _lib.Problem()
        p.feat = self.feats.ctypes.data
        p.fref = self.fref.ctypes.data
        p.pts3d = self.pts3d.ctypes.data
        p.Hf, p.Wf = self.feats.shape[0], self.feats.shape[1]
        p.cstride = self.feats.shape[-1]
        p.c_begin = int(self.c_begin)
        p.c_end = int(self.C if self.c_end is None else min(self.c_end, self.C))
        p.ld_ref = self.fref.shape[1]
        p.N = self.pts3d.shape[0]
        p.im_width, p.im_height = int(self.im_width), int(self.im_height)
        p.K[:] = list(np.asarray(self.K, dtype=np.float64).reshape(9))
        p.R0[:] = list(np.asarray(self.R0, dtype=np.float64).reshape(9))
        p.t0[:] = list(np.asarray(self.t0, dtype=np.float64).reshape(3))
        return p


def problem_host(feats, fref, pts3d, K, im_width, im_height, R0, t0, C=None, c_begin=0, c_end=None, layout=None):
    """One problem over host buffers (pack_host's map, fref [N, C] cast to the map's dtype and
    padded to its channel stride, pts3d [N, 3] fp64)."""
    layout = layout or ("f" if feats.ndim == 3 else "fgrad")
    cs = feats.shape[-1]
    fref = np.asarray(fref)
    C = fref.shape[1] if C is None else C
    fr = np.zeros((fref.shape[0], cs), dtype=feats.dtype)
    fr[:, :fref.shape[1]] = fref
    pts = np.ascontiguousarray(np.asarray(pts3d, dtype=np.float64).reshape(-1, 3))
    return HostProblem(np.ascontiguousarray(feats), layout, C, fr, pts, K, im_width, im_height, R0, t0, c_begin,
                       c_end)


def refine_cpu(problems, options, trace=False, n_threads=0, sobel_flags=0):
    """fmpnp_refine_batch_cpu over host problems: ([result dict], [trace dict] | None), the same
    dicts as fmpnp.refine.refine.  n_threads: host threads (0: every core)."""
    n = len(problems)
    if n == 0:
        return [], ([] if trace else None)
    lays = {p.layout for p in problems}
    dts = {p.feats.dtype for p in problems}
    if len(lays) > 1 or len(dts) > 1:
        raise ValueError("all problems of a call share one layout and dtype")
    o = _lib.Options.from_buffer_copy(options)
    o.layout = _lib.LAYOUT_F if lays.pop() == "f" else _lib.LAYOUT_FGRAD
    o.dtype = _lib.F64 if dts.pop() == np.float64 else _lib.F32
    if o.layout == _lib.LAYOUT_F:
        o.sobel_flags = int(sobel_flags)
    descs = (_lib.Problem * n)(*[p.descriptor() for p in problems])
    res = (_lib.Result * n)()
    stride = max(1, o.n_iters + 1) if trace else 0
    tr = (_lib.TraceEntry * (n * stride))() if trace else None
    rc = _lib.load().fmpnp_refine_batch_cpu(descs, n, ctypes.byref(o), res, tr, stride, int(n_threads))
    _lib.check(rc, "fmpnp_refine_batch_cpu")
    results = [_result_dict(r) for r in res]
    traces = None
    if trace:
        traces = [_trace_dict(tr[i * stride:(i + 1) * stride], results[i]["n_evals"]) for i in range(n)]
    return results, traces
