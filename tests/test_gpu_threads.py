"""The synchronous entry points' threading contract ("one call per stream,
thread-safe across distinct streams and devices"; 8e: one host thread per device).

fmpnp_refine_batch and fmpnp_feature_pnp keep their scratch per (device, stream)
(csrc/fmpnp_internal.h StreamScratch), so two host threads on two streams of one device run
their calls concurrently: results bit-identical to serial calls, and a wall time below the
serial one (the launches of the two streams overlap on the device).  Calls on ONE stream from
two threads serialise on that stream's scratch and stay correct."""
import threading
import time
from collections import namedtuple

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import fmpnp  # noqa: E402
from fmpnp import _lib, refine as rf, synth  # noqa: E402

DEV = "cuda:0"
Pred = namedtuple("Prediction", "points_3d reference_inliers matrix quaternion reference_filename")


def _problems(B, seed0):
    out = []
    for q in range(B):
        inp = synth.problem_inputs(512, 256, 240, 320, seed=seed0 + q, device=DEV)
        feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=DEV)
        out.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                   inp["R0"], inp["t0"]))
    return out


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert np.array_equal(x["R"], y["R"]) and np.array_equal(x["t"], y["t"])
        assert x["best_cost"] == y["best_cost"] and x["n_evals"] == y["n_evals"] and x["status"] == y["status"]


def _in_threads(fns):
    out, errs = [None] * len(fns), []

    def run(i):
        try:
            out[i] = fns[i]()
        except BaseException as e:  # noqa: BLE001  (re-raised in the main thread)
            errs.append(e)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(fns))]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    wall = time.perf_counter() - t0
    if errs:
        raise errs[0]
    return out, wall


def _abi_call(probs, opts, stream):
    """One thread's calls of fmpnp_refine_batch through the C ABI (ctypes releases the GIL for the call):
    descriptors and result buffers built once, so the loop is the library's own work, not Python's."""
    import ctypes
    n = len(probs)
    descs = (_lib.Problem * n)(*[p.descriptor() for p in probs])
    o = rf.bind_layout(probs, opts)
    res = (_lib.Result * n)()
    sp = ctypes.c_void_p(stream.cuda_stream)
    L = _lib.load()

    def call(read=True):
        _lib.check(L.fmpnp_refine_batch(descs, n, ctypes.byref(o), res, None, 0, sp), "fmpnp_refine_batch")
        return [rf._result_dict(r) for r in res] if read else None
    return call


def test_refine_batch_two_streams_concurrent():
    """Two threads, one stream each, 12 calls of fmpnp_refine_batch each (96 queries per call: two
    calls fill 192 of the 256 CUs): bit-identical to the serial calls, and faster than them (the two
    streams' launches overlap on the device)."""
    B, reps = 96, 12
    pa, pb = _problems(B, 0), _problems(B, 1000)
    opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
    sa, sb = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    ca_, cb_ = _abi_call(pa, opts, sa), _abi_call(pb, opts, sb)

    def loop(call):
        def f():
            for _ in range(reps - 1):
                call(read=False)
            return call()
        return f
    # the reference results (and both streams' scratch warmed), then the serial time
    ra, rb = ca_(), cb_()
    with torch.cuda.stream(sa):
        base_a, _ = rf.refine(pa, opts)
    _same(ra, base_a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(ca_)()
    loop(cb_)()
    serial = time.perf_counter() - t0
    (la, lb), wall = _in_threads([loop(ca_), loop(cb_)])
    _same(la, ra)
    _same(lb, rb)
    print(f"fmpnp_refine_batch, 2 x {reps} calls of B={B}: serial {serial * 1e3:.1f} ms, two threads {wall * 1e3:.1f} ms")
    assert wall < 0.8 * serial, (wall, serial)


def test_refine_batch_one_stream_two_threads_serialise():
    """Two threads on the SAME stream: the calls serialise on the stream's scratch, results exact."""
    B = 16
    pa, pb = _problems(B, 50), _problems(B, 70)
    opts = rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
    s = torch.cuda.Stream(DEV)
    with torch.cuda.stream(s):
        ra, _ = rf.refine(pa, opts)
        rb, _ = rf.refine(pb, opts)

    def calls(probs):
        def f():
            with torch.cuda.stream(s):
                return [rf.refine(probs, opts)[0] for _ in range(6)]
        return f
    (la, lb), _ = _in_threads([calls(pa), calls(pb)])
    for r in la:
        _same(r, ra)
    for r in lb:
        _same(r, rb)


def _query(seed):
    (batch,), img = synth.pipeline_queries(1, 1, 512, 256, 240, 320, device=DEV, seed0=seed)
    q, r, p, K = batch[0]
    return q[None], r, Pred(p.points_3d, p.reference_inliers, p.matrix, np.array([1.0, 0, 0, 0]), "ref.png"), K, img


def test_feature_pnp_two_streams_concurrent():
    """fmpnp_feature_pnp (the consumer's one-call path) from two threads on two streams: each
    thread's poses and attributes equal its serial calls bit for bit."""
    qa, qb = _query(21), _query(22)
    sa, sb = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)

    def calls(args, stream, reps=8):
        def f():
            with torch.cuda.stream(stream):
                out = []
                for _ in range(reps):
                    m = fmpnp.sparseFeaturePnP(50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01)
                    R, t, m = fmpnp.feature_pnp(*args, model=m)
                    out.append((R, t, float(m.best_cost_), m.best_num_inliers_))
                return out
        return f
    ra = calls(qa, sa, 1)()[0]
    rb = calls(qb, sb, 1)()[0]
    (la, lb), wall = _in_threads([calls(qa, sa), calls(qb, sb)])
    for got, ref in ((la, ra), (lb, rb)):
        for R, t, c, n in got:
            assert torch.equal(R, ref[0]) and torch.equal(t, ref[1]) and c == ref[2] and n == ref[3]
    print(f"fmpnp_feature_pnp, 2 threads x 8 calls: {wall * 1e3:.1f} ms")
