"""The launch planner, validation and workspace sizing of libfmpnp.so on the host, without a GPU
(FMPNP_PLAN_CUS gives the planner a CU count; the occupancy query then answers one block per CU).

These are the host paths of csrc/fmpnp_api.hip (make_plan, validate, fmpnp_workspace_size,
fmpnp_plan) that every launch runs before it touches the device; tools/sanitize.sh runs them
under ASan + UBSan.  Shapes: BASELINE.json configs[1..4] and the RobotCar pyramid."""
import ctypes

import pytest

from fmpnp import _lib, refine as rf

EINVAL, ETOOBIG = -1, -4


@pytest.fixture(autouse=True)
def _cus(monkeypatch):
    # (the library honours FMPNP_PLAN_CUS only without a device: on a host with one, the plans below --
    # sized for 256 CUs -- hold only on a 256-CU device)
    import torch
    if torch.cuda.is_available() and torch.cuda.get_device_properties(0).multi_processor_count != 256:
        pytest.skip("the planner plans for the device present, which does not have 256 CUs")
    monkeypatch.setenv("FMPNP_PLAN_CUS", "256")


def descs(n, N=512, C=256, Hf=240, Wf=320, cb=0, ce=None, im=(1280, 960), window=False):
    arr = (_lib.Problem * max(n, 1))()
    cs = (C + 3) // 4 * 4
    for i in range(n):
        p = arr[i]
        p.feat, p.fref, p.pts3d = 0x1000, 0x2000, 0x3000  # never dereferenced by the planner
        p.Hf, p.Wf, p.cstride, p.c_begin, p.c_end, p.ld_ref, p.N = Hf, Wf, cs, cb, C if ce is None else ce, cs, N
        p.im_width, p.im_height = im
        p.K[:] = [1000.0, 0, 640.0, 0, 1000.0, 480.0, 0, 0, 1]
        p.R0[:] = [1.0, 0, 0, 0, 1.0, 0, 0, 0, 1.0]
        p.window = 0x4000 if window else None
    return arr


def plan(n, opts, **kw):
    return _lib.plan(descs(n, **kw), n, opts)


def rc_of(n, opts, **kw):
    info = _lib.LaunchInfo()
    return _lib.load().fmpnp_plan(descs(n, **kw), n, ctypes.byref(opts), ctypes.byref(info))


def ws(n, opts, **kw):
    return _lib.load().fmpnp_workspace_size(descs(n, **kw), n, ctypes.byref(opts))


GM = dict(n_iters=50, lambda0=0.01, loss=_lib.GEMAN_MCCLURE, dtype=_lib.F32)


def test_headline_plan():
    """configs[2]'s per-GPU 128 queries: one latency workgroup per query with the speculative
    gathers, no helpers (no two spare CUs per problem)."""
    i = plan(128, rf.make_options(**GM))
    assert (i["wgs_per_problem"], i["grid"], i["build_name"], i["variant_name"], i["helpers"], i["team"]) == \
        (1, 128, "latency", "GM_SPEC_512", 0, 0)
    assert i["lds_bytes"] <= 160 * 1024


def test_single_query_takes_helpers():
    i = plan(1, rf.make_options(**GM))
    assert i["wgs_per_problem"] == 1 and i["helpers"] >= 2 and i["variant_name"] == "GM_SPEC_H_512"
    i = plan(1, rf.make_options(**GM), N=448)  # (fewer than 449 points: the runtime carve)
    assert i["variant_name"] == "GM_SPEC_H"


def test_two_per_cu_takes_the_throughput_build():
    i = plan(1024, rf.make_options(**GM))
    assert (i["build_name"], i["variant_name"], i["wgs_per_problem"], i["speculate"]) == ("throughput", "GM", 1, 0)
    # more problems than CUs (but fewer than two per CU): the throughput build too -- the latency build
    # would run a second round of workgroups (profiles/r05_wps_mid_batch.txt); one per CU stays latency
    i = plan(384, rf.make_options(**GM))
    assert (i["build_name"], i["variant_name"]) == ("throughput", "GM")
    i = plan(256, rf.make_options(**GM))
    assert (i["build_name"], i["variant_name"]) == ("latency", "GM_SPEC_512")


def test_ratio_and_variants():
    i = plan(128, rf.make_options(ratio_threshold=0.8, **GM))
    assert i["ratio"] == 1 and i["variant_name"] == "GM_SPEC_512"
    i = plan(128, rf.make_options(**dict(GM, dtype=_lib.F64)), C=128)  # (the 512-point carve: fp32 texels only)
    assert i["variant_name"] == "GM_SPEC"
    i = plan(128, rf.make_options(**GM), N=449)
    assert i["variant_name"] == "GM_SPEC_512"
    i = plan(128, rf.make_options(**GM), N=448)
    assert i["variant_name"] == "GM_SPEC"
    i = plan(128, rf.make_options(**dict(GM, loss=_lib.CAUCHY)))
    assert i["variant_name"] == "NEAREST_SPEC"
    i = plan(128, rf.make_options(sampling="bilinear", **GM))
    assert (i["build_name"], i["variant_name"]) == ("wide", "BILINEAR") and i["wgs_per_problem"] >= 2
    o = rf.make_options(**GM)
    o.layout = _lib.LAYOUT_F
    i = plan(1, o)
    assert i["variant_name"] == "F_GM" and i["wgs_per_problem"] > 1 and i["team"] == 1


@pytest.mark.parametrize("N,C,Hf,Wf", [(2048, 512, 480, 640), (866, 1024, 256, 256), (64, 3, 120, 160)])
def test_large_and_toy_problems_plan(N, C, Hf, Wf):
    for n in (1, 32, 128):
        i = plan(n, rf.make_options(**GM), N=N, C=C, Hf=Hf, Wf=Wf, im=(4 * Wf, 4 * Hf))
        assert i["lds_bytes"] <= 160 * 1024 and i["grid"] >= n * i["wgs_per_problem"] // max(1, i["teams"] // n or 1)
        assert ws(n, rf.make_options(**GM), N=N, C=C, Hf=Hf, Wf=Wf, im=(4 * Wf, 4 * Hf)) >= 0


def test_workspace_grows_with_teams():
    one = ws(1, rf.make_options(**dict(GM, wgs_per_problem=8)))
    many = ws(64, rf.make_options(**dict(GM, wgs_per_problem=8)))
    assert 0 < one < many


def test_validation_errors():
    o = rf.make_options(**GM)
    assert rc_of(1, o, N=-1) == EINVAL
    assert rc_of(1, o, cb=8, ce=4) == EINVAL            # c_end < c_begin
    assert rc_of(1, o, C=256, ce=300) == EINVAL          # c_end beyond the stride
    assert rc_of(1, o, im=(1 << 24, 960)) == ETOOBIG     # x * Wf overflows 32 bits
    bad = rf.make_options(**GM)
    bad.dtype = 7
    assert rc_of(1, bad) == EINVAL
    bad = rf.make_options(**dict(GM, dtype=_lib.F64))
    bad.layout = _lib.LAYOUT_F                           # the f-only layout is fp32 only
    assert rc_of(1, bad) == EINVAL
    bad = rf.make_options(**GM)
    bad.sobel_flags = 4
    assert rc_of(1, bad) == EINVAL
    d = descs(1)
    d[0].feat = 0
    info = _lib.LaunchInfo()
    assert _lib.load().fmpnp_plan(d, 1, ctypes.byref(o), ctypes.byref(info)) == EINVAL


def test_windowed_problems_plan_one_workgroup(monkeypatch):
    """A packed window (fmpnp_problem.window) on the f-only layout forces one workgroup per problem
    (a window miss stops the problem inside its workgroup); on the packed f/gx/gy planes a miss is
    only flagged, so the plan keeps its workgroups but drops the speculative gathers (they would read
    predicted texels outside the window) and takes the variant with the window check (_W); bilinear
    sampling refuses windows."""
    o = rf.make_options(**GM)
    o.layout = _lib.LAYOUT_F
    i = plan(1, o)
    assert i["wgs_per_problem"] > 1  # (a single f-only problem spreads over CUs)
    i = plan(1, o, window=True)
    assert i["wgs_per_problem"] == 1 and i["team"] == 0
    i = plan(128, rf.make_options(**GM))
    assert i["speculate"] == 1 and i["variant_name"] == "GM_SPEC_512"
    i = plan(128, rf.make_options(**GM), window=True)
    assert i["speculate"] == 0 and i["variant_name"] == "GM_W" and i["build_name"] == "latency"
    i = plan(1, rf.make_options(**GM), window=True)  # (one problem: the first-evaluation helpers too)
    assert i["variant_name"] in ("GM_W", "GM_H_W")
    i = plan(512, rf.make_options(**GM), window=True)  # (no throughput build: it has no _W variant)
    assert i["variant_name"] == "GM_W" and i["build_name"] == "latency"
    i = plan(512, rf.make_options(**GM))
    assert i["variant_name"] == "GM" and i["build_name"] == "throughput"
    with pytest.raises(_lib.FmpnpError):
        plan(1, rf.make_options(**dict(GM, sampling="bilinear")), window=True)
