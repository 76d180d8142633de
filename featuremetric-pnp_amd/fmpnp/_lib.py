"""ctypes binding of libfmpnp.so (include/fmpnp.h).

The library is the only compute path of this package: if it is missing, or no
gfx950 device is visible, every entry point raises -- there is no CPU fallback.
torch is imported first so that the process has exactly one HIP runtime
(libamdhip64.so.7 is shared by SONAME with torch's bundled copy).
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before libfmpnp)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FMPNP_LIB_PATH") or os.path.join(HERE, "lib", "libfmpnp.so")  # override: A/B builds

# enums / constants (include/fmpnp.h)
SQUARED, HUBER, CAUCHY, GEMAN_MCCLURE, BARRON = 0, 1, 2, 3, 4
NEAREST, BILINEAR = 0, 1
LAYOUT_FGRAD, LAYOUT_F = 0, 1
F32, F64 = 0, 1
MODE_FORWARD, MODE_COMPUTE_COST = 0, 1
STATUS_OK, STATUS_NO_SUPPORT, STATUS_NAN, STATUS_NO_SUPPORT_TRIAL, STATUS_SYNC_TIMEOUT = 0, 1, 2, 4, 8
STATUS_HELPER_WAIT = 16  # informational: a first-evaluation helper did not publish in time (results unaffected)
STATUS_WINDOW = 32  # a point left its packed window (fmpnp_pack_features_f_window_batch): result invalid, re-run
ABI_VERSION = 4
# LM kernel builds and variants (fmpnp_launch_info)
BUILD_WIDE, BUILD_LATENCY, BUILD_THROUGHPUT = 1, 2, 4
BUILD_NAMES = {BUILD_WIDE: "wide", BUILD_LATENCY: "latency", BUILD_THROUGHPUT: "throughput"}
VARIANT_NAMES = ["NEAREST", "GM", "BILINEAR", "F_NEAREST", "F_GM", "BIL_DIRECT", "GM_SPEC", "NEAREST_SPEC",
                 "GM_SPEC_H", "NEAREST_SPEC_H", "GM_H", "NEAREST_H", "GM_SPEC_512", "GM_SPEC_H_512", "GM_W", "NEAREST_W",
                 "GM_H_W", "NEAREST_H_W"]
ERRORS = {-1: "EINVAL", -2: "EALIGN", -3: "ENOMEM", -4: "ETOOBIG", -5: "ENODEV", -6: "ERANGE"}
ERANGE = -6  # fmpnp_feature_pnp: a reference inlier outside the reference map (IndexError)


class Options(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("n_iters", ctypes.c_int), ("lambda0", ctypes.c_double),
                ("use_ratio", ctypes.c_int), ("ratio_threshold", ctypes.c_double), ("loss", ctypes.c_int),
                ("barron_alpha", ctypes.c_double), ("sampling", ctypes.c_int), ("dtype", ctypes.c_int),
                ("wgs_per_problem", ctypes.c_int), ("max_teams", ctypes.c_int), ("no_memo", ctypes.c_int),
                ("layout", ctypes.c_int), ("sobel_flags", ctypes.c_int), ("helpers", ctypes.c_int)]


class Problem(ctypes.Structure):
    _fields_ = [("feat", ctypes.c_void_p), ("fref", ctypes.c_void_p), ("pts3d", ctypes.c_void_p),
                ("Hf", ctypes.c_int), ("Wf", ctypes.c_int), ("cstride", ctypes.c_int), ("c_begin", ctypes.c_int),
                ("c_end", ctypes.c_int), ("ld_ref", ctypes.c_int), ("N", ctypes.c_int),
                ("im_width", ctypes.c_int), ("im_height", ctypes.c_int),
                ("K", ctypes.c_double * 9), ("R0", ctypes.c_double * 9), ("t0", ctypes.c_double * 3),
                ("window", ctypes.c_void_p)]


class Level(ctypes.Structure):
    _fields_ = [("c_begin", ctypes.c_int), ("c_end", ctypes.c_int)]


class Result(ctypes.Structure):
    _fields_ = [("R", ctypes.c_double * 9), ("t", ctypes.c_double * 3), ("initial_cost", ctypes.c_double),
                ("best_cost", ctypes.c_double), ("final_lambda", ctypes.c_double), ("final_lr", ctypes.c_double),
                ("best_num_inliers", ctypes.c_int), ("n_evals", ctypes.c_int), ("n_steps", ctypes.c_int),
                ("n_accepted", ctypes.c_int), ("status", ctypes.c_int), ("has_best", ctypes.c_int),
                ("texel_gathers", ctypes.c_longlong)]


class TraceEntry(ctypes.Structure):
    _fields_ = [("R", ctypes.c_double * 9), ("t", ctypes.c_double * 3), ("cost", ctypes.c_double),
                ("lambda_after", ctypes.c_double), ("lr_after", ctypes.c_double), ("n_supported", ctypes.c_int),
                ("n_kept", ctypes.c_int), ("accepted", ctypes.c_int)]


class LaunchInfo(ctypes.Structure):
    _fields_ = [("teams", ctypes.c_int), ("wgs_per_problem", ctypes.c_int), ("grid", ctypes.c_int),
                ("lds_bytes", ctypes.c_int), ("build", ctypes.c_int), ("variant", ctypes.c_int),
                ("team", ctypes.c_int), ("ratio", ctypes.c_int), ("dtype", ctypes.c_int), ("helpers", ctypes.c_int),
                ("speculate", ctypes.c_int)]


EXPORTS = ["fmpnp_abi_version", "fmpnp_build_info", "fmpnp_device_check", "fmpnp_pack_features",
           "fmpnp_gather_reference", "fmpnp_gather_reference_async", "fmpnp_pack_features_batch", "fmpnp_pack_features_f",
           "fmpnp_gather_reference_batch", "fmpnp_workspace_size", "fmpnp_refine_batch_async", "fmpnp_refine_batch",
           "fmpnp_last_launch", "fmpnp_debug_stamps", "fmpnp_plan", "fmpnp_last_launch_info",
           "fmpnp_pack_features_f_window_batch", "fmpnp_feature_pnp", "fmpnp_compute_cost_async",
           "fmpnp_feature_pnp_reruns", "fmpnp_refine_batch_cpu"]

_LIB = None


class FmpnpError(RuntimeError):
    pass


def load():
    """Load libfmpnp.so (no device needed to load it)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise FmpnpError(f"libfmpnp.so not built ({LIB_PATH}); run `python -c 'import __graft_entry__ as g; "
                         f"g.build()'` or `make -C featuremetric-pnp_amd`")
    L = ctypes.CDLL(LIB_PATH)
    vp, i, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    L.fmpnp_abi_version.restype = i
    L.fmpnp_build_info.restype = ctypes.c_char_p
    L.fmpnp_device_check.argtypes = [i]
    L.fmpnp_device_check.restype = i
    L.fmpnp_pack_features.argtypes = [vp, vp, vp, i, i, i, i, vp, i, i, i, i, vp]
    L.fmpnp_pack_features.restype = i
    L.fmpnp_gather_reference.argtypes = [vp, i, i, i, i, vp, i, i, i, vp, i, i, vp]
    L.fmpnp_gather_reference.restype = i
    L.fmpnp_gather_reference_async.argtypes = [vp, i, i, i, i, vp, i, i, i, vp, i, i, vp, vp]
    L.fmpnp_gather_reference_async.restype = i
    L.fmpnp_pack_features_batch.argtypes = [i, vp, vp, vp, i, i, i, i, i, vp]
    L.fmpnp_pack_features_f.argtypes = [vp, i, i, i, i, vp, i, i, vp]
    L.fmpnp_pack_features_f.restype = i
    L.fmpnp_pack_features_batch.restype = i
    L.fmpnp_gather_reference_batch.argtypes = [i, vp, vp, vp, vp, i, i, vp, vp, i, i, vp, vp]
    L.fmpnp_gather_reference_batch.restype = i
    L.fmpnp_pack_features_f_window_batch.argtypes = [vp, vp, i, vp, i, i, vp]
    L.fmpnp_pack_features_f_window_batch.restype = i
    L.fmpnp_point_costs.argtypes = [ctypes.POINTER(Problem), i, i, vp, vp, vp]
    L.fmpnp_point_costs.restype = i
    L.fmpnp_workspace_size.argtypes = [ctypes.POINTER(Problem), i, ctypes.POINTER(Options)]
    L.fmpnp_workspace_size.restype = ctypes.c_size_t
    L.fmpnp_refine_batch_async.argtypes = [vp, ctypes.POINTER(Problem), i, i, ctypes.POINTER(Options), vp, vp, i, vp,
                                           ctypes.c_size_t, vp]
    L.fmpnp_refine_batch_async.restype = i
    L.fmpnp_refine_batch.argtypes = [ctypes.POINTER(Problem), i, ctypes.POINTER(Options), ctypes.POINTER(Result),
                                     ctypes.POINTER(TraceEntry), i, vp]
    L.fmpnp_refine_batch.restype = i
    if hasattr(L, "fmpnp_refine_batch_cpu"):  # (A/B builds of earlier sources lack it)
        L.fmpnp_refine_batch_cpu.argtypes = [ctypes.POINTER(Problem), i, ctypes.POINTER(Options),
                                             ctypes.POINTER(Result), ctypes.POINTER(TraceEntry), i, i]
        L.fmpnp_refine_batch_cpu.restype = i
    L.fmpnp_last_launch.argtypes = [ctypes.POINTER(i)] * 4
    L.fmpnp_last_launch.restype = i
    L.fmpnp_plan.argtypes = [ctypes.POINTER(Problem), i, ctypes.POINTER(Options), ctypes.POINTER(LaunchInfo)]
    L.fmpnp_plan.restype = i
    L.fmpnp_last_launch_info.argtypes = [ctypes.POINTER(LaunchInfo)]
    L.fmpnp_last_launch_info.restype = i
    L.fmpnp_compute_cost_async.argtypes = [ctypes.POINTER(Problem), i, i, i, d, vp, vp, vp, vp]
    L.fmpnp_compute_cost_async.restype = i
    dp = ctypes.POINTER(ctypes.c_double)
    L.fmpnp_feature_pnp.argtypes = [vp, i, i, i, i, vp, i, i, i, i, vp, vp, i, dp, dp, dp, i, i,
                                    ctypes.POINTER(Level), i, ctypes.POINTER(Options), i, vp, vp, i, vp]
    L.fmpnp_feature_pnp.restype = i
    if hasattr(L, "fmpnp_feature_pnp_reruns"):  # (A/B builds of earlier sources lack it)
        L.fmpnp_feature_pnp_reruns.restype = ctypes.c_longlong
    if L.fmpnp_abi_version() != ABI_VERSION:
        raise FmpnpError("libfmpnp ABI mismatch")
    _LIB = L
    return L


def check(rc, what):
    if rc != 0:
        name = ERRORS.get(rc, f"hipError {rc}")
        raise FmpnpError(f"{what} failed: {name}")


_DEVICE_OK = {}


def require_device(device):
    """The HIP path needs a gfx950 device; anything else is a hard error."""
    if not torch.cuda.is_available():
        raise FmpnpError("fmpnp needs an AMD MI355X (gfx950) GPU; none is visible (no CPU fallback)")
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    if idx not in _DEVICE_OK:
        rc = load().fmpnp_device_check(idx)
        if rc != 0:
            raise FmpnpError(f"device {idx} is not a gfx950 (fmpnp_device_check -> {rc})")
        _DEVICE_OK[idx] = True
    return idx


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def spec_build():
    """True when libfmpnp.so has the speculative next-texel gathers compiled in (the default;
    a -DFMPNP_SPEC=0 build leaves them out).  Per launch, fmpnp_options.no_memo = 2 turns them off."""
    return b"speculative_gathers=1" in load().fmpnp_build_info()


def _info_dict(info):
    d = {name: getattr(info, name) for name, _ in LaunchInfo._fields_}
    d["build_name"] = BUILD_NAMES.get(info.build, str(info.build))
    d["variant_name"] = VARIANT_NAMES[info.variant] if 0 <= info.variant < len(VARIANT_NAMES) else str(info.variant)
    d["dtype_name"] = "f64" if info.dtype == F64 else "f32"
    return d


from .build_id import kernel_name, source_digest  # noqa: E402,F401  (profile matching: bench.py)


def library_digest():
    """The source digest compiled into the loaded libfmpnp.so ("unknown" outside the Makefile)."""
    info = load().fmpnp_build_info().decode()
    return info.split("source_digest=", 1)[1].split(";")[0].strip() if "source_digest=" in info else "unknown"


def last_launch():
    """Plan of this thread's last LM launch: geometry, build, kernel variant, helpers."""
    info = LaunchInfo()
    load().fmpnp_last_launch_info(ctypes.byref(info))
    return _info_dict(info)


def plan(descs, n, options):
    """The launch plan (as last_launch()) for n fmpnp_problem descriptors and options, without
    launching (needs the device)."""
    info = LaunchInfo()
    check(load().fmpnp_plan(descs, n, ctypes.byref(options), ctypes.byref(info)), "fmpnp_plan")
    return _info_dict(info)
