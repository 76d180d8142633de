"""Batched preparation entry points (fmpnp_pack_features_batch, fmpnp_gather_reference_batch)
against the single-map ones on maps of different shapes, including channel counts that need
padding and an out-of-map reference inlier (the reference's IndexError,
optimize_feature_pnp.py:56)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_batched_pack_and_gather_equal_single_calls():
    import torch
    from fmpnp import _lib, refine as rf
    dev = torch.device("cuda", 0)
    L = _lib.load()
    vp = ctypes.c_void_p
    g = torch.Generator().manual_seed(11)
    shapes = [(37, 20, 28), (64, 33, 40), (5, 9, 13)]        # C, H, W (C = 37, 5: padded cstride)
    maps = [torch.randn(s, generator=g).to(dev) for s in shapes]
    single = [rf.pack_features(m, storage=torch.float32, device=dev).buf for m in maps]
    outs = [torch.zeros_like(b) for b in single]
    shape_arr = (ctypes.c_int * 12)(*[v for (C, H, W), b in zip(shapes, single) for v in (C, H, W, b.shape[3])])
    rc = L.fmpnp_pack_features_batch(3, (vp * 3)(*[m.data_ptr() for m in maps]),
                                     (vp * 3)(*[o.data_ptr() for o in outs]), shape_arr, _lib.F32, _lib.F32, 0, 0,
                                     _lib.LAYOUT_FGRAD, _lib.stream_ptr(dev))
    _lib.check(rc, "pack batch")
    torch.cuda.synchronize()
    for a, b in zip(single, outs):
        assert torch.equal(a, b)
    # reference gathers: square maps (the reference swaps the H / W scales), image 64 x 64
    refs = [torch.randn((C, 16, 16), generator=g).to(dev) for C in (37, 64, 5)]
    rng = np.random.default_rng(3)
    inls = [rng.uniform(0, 64, (n, 2)) for n in (10, 25, 7)]
    inls[2][4] = (500.0, 3.0)                                # query 2: one inlier off the map
    cs = [b.shape[3] for b in single]
    expect = []
    for i in range(3):
        if i == 2:
            with pytest.raises(IndexError):
                rf.gather_reference(refs[i], inls[i], (64, 64), cstride=cs[i])
            e = torch.zeros(1, dtype=torch.int32, device=dev)
            expect.append(rf.gather_reference(refs[i], inls[i], (64, 64), cstride=cs[i], err_flag=e))
        else:
            expect.append(rf.gather_reference(refs[i], inls[i], (64, 64), cstride=cs[i]))
    d_inl = [torch.from_numpy(a).to(dev) for a in inls]
    got = [torch.zeros_like(e) for e in expect]
    err = torch.zeros(3, dtype=torch.int32, device=dev)
    rc = L.fmpnp_gather_reference_batch(
        3, (vp * 3)(*[r.data_ptr() for r in refs]), (ctypes.c_int * 9)(*[v for r in refs for v in r.shape]),
        (vp * 3)(*[a.data_ptr() for a in d_inl]), (ctypes.c_int * 3)(10, 25, 7), 64, 64,
        (vp * 3)(*[o.data_ptr() for o in got]), (ctypes.c_int * 3)(*cs), _lib.F32, _lib.F32, vp(err.data_ptr()),
        _lib.stream_ptr(dev))
    _lib.check(rc, "gather batch")
    torch.cuda.synchronize()
    for a, b in zip(expect, got):
        assert torch.equal(a, b)
    assert err.tolist() == [0, 0, 1]


def test_batched_gather_with_empty_items_and_more_than_one_launch():
    """40 items (two launches of the item table) with empty ones among them: every
    non-empty item equals its single-call gather, empty items leave their flag at 0."""
    import torch
    from fmpnp import _lib, refine as rf
    dev = torch.device("cuda", 0)
    L = _lib.load()
    vp = ctypes.c_void_p
    g = torch.Generator().manual_seed(5)
    rng = np.random.default_rng(6)
    n = 40
    refs = [torch.randn((16, 12, 12), generator=g).to(dev) for _ in range(n)]
    counts = [0 if i % 7 == 3 else int(rng.integers(1, 20)) for i in range(n)]
    inls = [torch.from_numpy(rng.uniform(0, 48, (max(c, 1), 2))).to(dev) for c in counts]
    outs = [torch.zeros((max(c, 1), 16), device=dev) for c in counts]
    err = torch.zeros(n, dtype=torch.int32, device=dev)
    rc = L.fmpnp_gather_reference_batch(
        n, (vp * n)(*[r.data_ptr() for r in refs]), (ctypes.c_int * (3 * n))(*[v for r in refs for v in r.shape]),
        (vp * n)(*[a.data_ptr() for a in inls]), (ctypes.c_int * n)(*counts), 48, 48,
        (vp * n)(*[o.data_ptr() for o in outs]), (ctypes.c_int * n)(*([16] * n)), _lib.F32, _lib.F32,
        vp(err.data_ptr()), _lib.stream_ptr(dev))
    _lib.check(rc, "gather batch")
    torch.cuda.synchronize()
    assert not err.any()
    for i in range(n):
        if counts[i] == 0:
            assert not outs[i].any()
            continue
        one = rf.gather_reference(refs[i], inls[i].cpu().numpy(), (48, 48), cstride=16)
        assert torch.equal(one, outs[i])



def test_batched_f_only_pack_equals_single_calls():
    """FMPNP_LAYOUT_F batch (one launch per 32 maps) against single-map f-only packs, on
    mixed shapes (padded channel counts zero-filled) across two launches."""
    import torch
    from fmpnp import _lib, refine as rf
    dev = torch.device("cuda", 0)
    L = _lib.load()
    vp = ctypes.c_void_p
    g = torch.Generator().manual_seed(12)
    shapes = [(37, 20, 28), (64, 33, 40), (5, 9, 13), (256, 24, 32)] * 9   # 36 maps
    maps = [torch.randn(s, generator=g).to(dev) for s in shapes]
    single = [rf.pack_features(m, storage=torch.float32, device=dev, layout="f").buf for m in maps]
    outs = [torch.full_like(b, 7.0) for b in single]   # padding must be overwritten with zeros
    n = len(maps)
    shape_arr = (ctypes.c_int * (4 * n))(*[v for (C, H, W), b in zip(shapes, single) for v in (C, H, W, b.shape[2])])
    rc = L.fmpnp_pack_features_batch(n, (vp * n)(*[m.data_ptr() for m in maps]),
                                     (vp * n)(*[o.data_ptr() for o in outs]), shape_arr, _lib.F32, _lib.F32, 0, 0,
                                     _lib.LAYOUT_F, _lib.stream_ptr(dev))
    _lib.check(rc, "pack batch f")
    torch.cuda.synchronize()
    for a, b in zip(single, outs):
        assert torch.equal(a, b)
