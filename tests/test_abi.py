"""The C ABI (include/fmpnp.h): library loads without a GPU, exports every declared
entry point, and the ctypes mirror of every struct matches the C layout."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from fmpnp import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fmpnp.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w[\w\s\*]*?\b(fmpnp_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_abi():
    fns = declared_functions()
    for f in ("fmpnp_refine_batch", "fmpnp_refine_batch_async", "fmpnp_pack_features", "fmpnp_gather_reference",
              "fmpnp_workspace_size", "fmpnp_abi_version"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert not missing, missing
    assert L.fmpnp_abi_version() == _lib.ABI_VERSION == 4
    assert b"gfx950" in L.fmpnp_build_info()


def test_library_is_a_gfx950_code_object():
    """The fat binary embeds an amdgcn code object for gfx950 (and nothing else to fall back to)."""
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob


STRUCTS = {"fmpnp_options": _lib.Options, "fmpnp_problem": _lib.Problem, "fmpnp_result": _lib.Result,
           "fmpnp_trace_entry": _lib.TraceEntry, "fmpnp_launch_info": _lib.LaunchInfo, "fmpnp_level": _lib.Level}


@pytest.mark.parametrize("name", sorted(STRUCTS))
def test_struct_layout_matches_c(name):
    cls = STRUCTS[name]
    lines = [f'printf("%zu\\n", sizeof({name}));']
    for fname, _ in cls._fields_:
        lines.append(f'printf("%zu\\n", offsetof({name}, {fname}));')
    prog = "#include <stdio.h>\n#include <stddef.h>\n#include \"fmpnp.h\"\nint main(void){\n" + "\n".join(lines) + \
           "\nreturn 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        vals = [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(cls)
    for (fname, _), off in zip(cls._fields_, vals[1:]):
        assert getattr(cls, fname).offset == off, fname


def test_entry_points_reject_bad_arguments_without_a_device():
    """Argument validation happens before any device call: no GPU needed."""
    L = _lib.load()
    assert L.fmpnp_pack_features(None, None, None, 0, 1, 1, 1, None, 0, 1, 0, 0, None) == -1
    assert L.fmpnp_gather_reference(None, 0, 1, 1, 1, None, 1, 1, 1, None, 0, 1, None) == -1
    o = _lib.Options()
    o.dtype = 7
    assert L.fmpnp_refine_batch(None, 1, ctypes.byref(o), None, None, 0, None) == -1
    assert L.fmpnp_gather_reference_async(None, 0, 1, 1, 1, None, 1, 1, 1, None, 0, 1, None, None) == -1
    # batched forms: negative counts, missing arrays, and one bad item among good ones are
    # refused before anything is launched
    vp = ctypes.c_void_p
    assert L.fmpnp_pack_features_batch(-1, None, None, None, 0, 0, 0, 0, 0, None) == -1
    assert L.fmpnp_pack_features_batch(1, None, None, None, 0, 0, 0, 0, 0, None) == -1
    assert L.fmpnp_pack_features_batch(0, None, None, None, 0, 0, 0, 0, 0, None) == 0
    two = (vp * 2)(1, 2)
    shape = (ctypes.c_int * 8)(4, 2, 2, 4, 4, 2, 2, 3)  # item 1: cstride < C
    assert L.fmpnp_pack_features_batch(2, two, two, shape, 0, 0, 0, 0, 0, None) == -1
    assert L.fmpnp_pack_features_batch(0, None, None, None, 0, 0, 0, 0, 7, None) == -1  # unknown layout
    assert L.fmpnp_pack_features_f(None, 0, 1, 1, 1, None, 0, 1, None) == -1
    # the f-only layout is fp32 with nearest sampling
    # (option checks run before any problem or device access)
    pb, res = _lib.Problem(), _lib.Result()
    o = _lib.Options()
    o.layout, o.dtype = _lib.LAYOUT_F, _lib.F64
    assert L.fmpnp_refine_batch(ctypes.byref(pb), 1, ctypes.byref(o), ctypes.byref(res), None, 0, None) == -1
    o.dtype, o.sampling = _lib.F32, _lib.BILINEAR
    assert L.fmpnp_refine_batch(ctypes.byref(pb), 1, ctypes.byref(o), ctypes.byref(res), None, 0, None) == -1
    o.sampling, o.layout = _lib.NEAREST, 5
    assert L.fmpnp_refine_batch(ctypes.byref(pb), 1, ctypes.byref(o), ctypes.byref(res), None, 0, None) == -1
    assert L.fmpnp_gather_reference_batch(1, None, None, None, None, 1, 1, None, None, 0, 0, None, None) == -1
    # per-point costs: missing outputs, a bad channel range or layout are refused
    vpp = ctypes.c_void_p
    assert L.fmpnp_point_costs(None, 0, 0, None, None, None) == -1
    p = _lib.Problem()
    p.N, p.feat, p.fref, p.pts3d = 4, 16, 16, 16
    p.Hf = p.Wf = p.im_width = p.im_height = 8
    p.cstride, p.c_begin, p.c_end, p.ld_ref = 4, 0, 8, 8           # c_end > cstride
    assert L.fmpnp_point_costs(ctypes.byref(p), 0, 0, vpp(16), vpp(16), None) == -1
    p.c_end = 4
    assert L.fmpnp_point_costs(ctypes.byref(p), 3, 0, vpp(16), vpp(16), None) == -1  # unknown layout
    assert L.fmpnp_point_costs(ctypes.byref(p), _lib.LAYOUT_F, _lib.F64, vpp(16), vpp(16), None) == -1
    p.N = 0
    assert L.fmpnp_point_costs(ctypes.byref(p), 0, 0, vpp(16), vpp(16), None) == 0
    rshape = (ctypes.c_int * 6)(4, 2, 2, 4, 2, 2)
    n_in = (ctypes.c_int * 2)(3, -1)                    # item 1: negative point count
    ld = (ctypes.c_int * 2)(4, 4)
    assert L.fmpnp_gather_reference_batch(2, two, rshape, two, n_in, 8, 8, two, ld, 0, 0, vp(3), None) == -1


def test_tail_sincos_matches_libm():
    """The LM tail's polynomial sin/cos (fmpnp_device.h sincos_small / sincos_rr, which
    replace the library sincos in so3exp_map, helpers/utils.py:209-221) stay within a few
    eps of libm over 0..200 rad; non-finite angles give NaN.  Host build of the same code."""
    pkg = os.path.join(ROOT, "featuremetric-pnp_amd")
    subprocess.run(["make", "-s", "-C", pkg, "build/test_host_math"], check=True, timeout=300)
    r = subprocess.run([os.path.join(pkg, "build", "test_host_math")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_window_pack_rejects_bad_arguments_without_a_device():
    """fmpnp_pack_features_f_window_batch validates every descriptor before launching: a radius
    below 2, a missing window map or output, a channel slice not starting at 0."""
    L = _lib.load()
    vp = ctypes.c_void_p
    p = _lib.Problem()
    p.feat, p.fref, p.pts3d, p.window = 256, 256, 256, 4096
    p.Hf, p.Wf, p.cstride, p.c_begin, p.c_end, p.ld_ref, p.N = 8, 8, 4, 0, 4, 4, 3
    p.im_width, p.im_height = 32, 32
    chw = (vp * 1)(4096)
    assert L.fmpnp_pack_features_f_window_batch(256, ctypes.byref(p), 1, chw, 0, 1, None) == -1   # radius < 2
    assert L.fmpnp_pack_features_f_window_batch(256, ctypes.byref(p), -1, chw, 0, 3, None) == -1  # n < 0
    assert L.fmpnp_pack_features_f_window_batch(256, ctypes.byref(p), 1, chw, 5, 3, None) == -1   # dtype
    for field, bad in (("window", None), ("feat", None), ("c_begin", 1), ("cstride", 6)):
        q = _lib.Problem.from_buffer_copy(p)
        setattr(q, field, bad)
        assert L.fmpnp_pack_features_f_window_batch(256, ctypes.byref(q), 1, chw, 0, 3, None) == -1, field
    assert L.fmpnp_pack_features_f_window_batch(256, ctypes.byref(p), 0, chw, 0, 3, None) == 0      # nothing to do


def test_feature_pnp_call_rejects_bad_arguments_without_a_device():
    """fmpnp_feature_pnp (one query of feature_pnp per call) validates its arguments before any
    device call: missing maps or outputs, a reference map of another channel count, a bad level,
    a compute_cost mode, an unknown dtype."""
    import numpy as np
    L = _lib.load()
    vp = ctypes.c_void_p
    dp = ctypes.POINTER(ctypes.c_double)
    K = np.eye(3).reshape(-1)
    inl, pts = np.zeros((4, 2)), np.ones((4, 3))
    o = _lib.Options()
    res = (_lib.Result * 4)()

    def call(q=4096, C=8, Cr=8, lv=None, nlv=0, opt=o, res_=res, dq=0, N=4, win=0):
        arr = (_lib.Level * max(nlv, 1))(*(lv or []))
        return L.fmpnp_feature_pnp(vp(q) if q else None, dq, C, 16, 16, vp(4096), 0, Cr, 16, 16,
                                   vp(inl.ctypes.data), vp(pts.ctypes.data), N, K.ctypes.data_as(dp),
                                   K.ctypes.data_as(dp), K[:3].ctypes.data_as(dp), 64, 64,
                                   arr if nlv else None, nlv, ctypes.byref(opt), win, res_, None, 0, None)
    assert call(q=0) == -1                                   # no query map
    assert call(Cr=9) == -1                                  # reference map of another channel count
    assert call(dq=3) == -1                                  # unknown dtype
    assert call(N=-1) == -1
    assert call(lv=[_lib.Level(0, 9)], nlv=1) == -1          # level beyond the map's channels
    assert call(lv=[_lib.Level(4, 4)], nlv=1) == -1          # empty level
    assert call(res_=None) == -1
    oc = _lib.Options.from_buffer_copy(o)
    oc.mode = _lib.MODE_COMPUTE_COST
    assert call(opt=oc) == -1                                # forward only (compute_cost runs inside)
    assert call(win=-1) == -1                                # a negative window radius
    of = _lib.Options.from_buffer_copy(o)
    of.layout = _lib.LAYOUT_F
    assert call(opt=of, win=5) == -1                         # windows: the packed f, gx, gy planes only
