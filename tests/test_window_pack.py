"""Windowed f-only packs (fmpnp_pack_features_f_window_batch, fmpnp.pipeline window=r).

The refinement reads only the 3x3 neighbourhoods of the texels its points visit
(featurePnP/model.py:303-311 projection, :74-97 indexing_), so the pipeline may pack only the
texels near each point's texel at the initial pose (optimize_feature_pnp.py:57-61 packs all of
them).  The LM kernel checks every gather against the window's plane 1 and stops a problem that
leaves it (FMPNP_STATUS_WINDOW); the pipeline packs such queries in full and refines them again.

Checked here: the packed texels equal the full pack's, plane 1 lies inside plane 0 and holds
every supported point's initial texel; the windowed pipeline's results equal the fully packed
pipeline's bit for bit on the easy and the hard start, including radii small enough that many
queries leave their window and take the refill.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402

import fmpnp  # noqa: E402
from fmpnp import _lib, refine as rf, synth  # noqa: E402  (no skip: a missing HIP library must fail)
from fmpnp.pipeline import RefinePipeline  # noqa: E402

DEV = torch.device("cuda", 0)


def _initial_texels(X, K, R, t, W, H, Hf, Wf):
    Pc = X @ R.T + t
    u = Pc @ K.T
    px, py = np.rint(u[:, 0] / u[:, 2]) - 1.0, np.rint(u[:, 1] / u[:, 2]) - 1.0
    ok = (px >= 0) & (px < W) & (py >= 0) & (py < H)
    row = (py[ok].astype(np.int64) * Hf) // H
    col = (px[ok].astype(np.int64) * Wf) // W
    return row, col


# (Wf = 43: no 16-byte column quads, the per-texel loads and window reads; fp64 CHW input: the converting
# loads; Hf = 30: a last tile of two rows; C = 37: a partial channel tile and a zero-padded stride)
@pytest.mark.parametrize("radius,Wf_,dt", [(2, 44, "f32"), (5, 44, "f32"), (2, 43, "f32"), (5, 44, "f64"),
                                           (2, 43, "f64")])
def test_window_pack_writes_exactly_the_marked_texels(radius, Wf_, dt):
    batches, (W, H) = synth.pipeline_queries(1, 3, N=200, C=37, Hf=30, Wf=Wf_, device=DEV, seed0=70)
    qs = batches[0]
    if dt == "f64":
        qs = [(a.double(), b, p, k) for (a, b, p, k) in qs]
    n = len(qs)
    C, Hf, Wf = qs[0][0].shape
    cs = (C + 3) // 4 * 4
    full = [rf.pack_features(q[0], storage=torch.float32, device=DEV, layout="f").buf for q in qs]
    outs = [torch.full((Hf, Wf, cs), float("nan"), device=DEV) for _ in range(n)]
    wins = [torch.full((2, Hf, Wf), 7, dtype=torch.uint8, device=DEV) for _ in range(n)]
    pts = [torch.as_tensor(np.asarray(q[2].points_3d), dtype=torch.float64, device=DEV) for q in qs]
    desc = np.zeros(n, dtype=rf.PROBLEM_DTYPE)
    desc["feat"] = [o.data_ptr() for o in outs]
    desc["fref"] = desc["feat"]
    desc["pts3d"] = [p.data_ptr() for p in pts]
    desc["window"] = [w.data_ptr() for w in wins]
    desc["Hf"], desc["Wf"], desc["cstride"], desc["c_end"], desc["ld_ref"] = Hf, Wf, cs, C, cs
    desc["N"] = [p.shape[0] for p in pts]
    desc["im_width"], desc["im_height"] = W, H
    desc["K"] = np.stack([np.asarray(q[3], np.float64).reshape(9) for q in qs])
    desc["R0"] = np.stack([np.asarray(q[2].matrix)[:3, :3].reshape(9) for q in qs])
    desc["t0"] = np.stack([np.asarray(q[2].matrix)[:3, 3] for q in qs])
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(DEV)
    vp = ctypes.c_void_p
    rc = _lib.load().fmpnp_pack_features_f_window_batch(
        vp(d_desc.data_ptr()), vp(desc.ctypes.data), n, (vp * n)(*[q[0].data_ptr() for q in qs]),
        _lib.F64 if dt == "f64" else _lib.F32, radius,
        _lib.stream_ptr(DEV))
    _lib.check(rc, "window pack")
    torch.cuda.synchronize()
    for i, q in enumerate(qs):
        w = wins[i].cpu().numpy()
        assert set(np.unique(w)) <= {0, 1}
        assert not (w[1] & ~w[0]).any()  # plane 1 (3x3 neighbourhood packed) inside plane 0
        T = np.asarray(q[2].matrix)
        row, col = _initial_texels(np.asarray(q[2].points_3d), np.asarray(q[3]), T[:3, :3], T[:3, 3], W, H, Hf, Wf)
        assert len(row) > 100 and w[1][row, col].all()
        # interior of plane 1: the whole 3x3 neighbourhood (clipped to the map) is in plane 0
        for y, x in zip(*np.nonzero(w[1])):
            assert w[0][max(y - 1, 0):y + 2, max(x - 1, 0):x + 2].all()
        m = torch.from_numpy(w[0].astype(bool)).to(DEV)
        assert torch.equal(outs[i][m], full[i][m])           # packed texels: the full pack's bits
        assert torch.isnan(outs[i][~m]).all()                # nothing else written
        assert 0.05 < w[0].mean() < 1.0


def _queries(init, nb, qb, seed0):
    batches, img = synth.pipeline_queries(nb, qb, 512, 256, 240, 320, device=DEV, seed0=seed0)
    if init != "easy":
        R0, t0 = synth.INITS[init]
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = R0, t0
        batches = [[(a, b, p._replace(matrix=T), k) for (a, b, p, k) in qs] for qs in batches]
    return batches, img


def _pipe(img, window):
    return RefinePipeline(img, storage=torch.float32, depth=2, window=window,
                          model_kwargs=dict(n_iters=50, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01,
                                            ratio_threshold=None))


@pytest.mark.parametrize("init", ["easy", "hard"])
def test_windowed_pipeline_equals_full_pack(init):
    """window = 6 (the bench's radius) and window = 2 (most queries leave it and are refilled):
    every query's result equals the fully packed pipeline's bit for bit."""
    batches, img = _queries(init, 2, 12, 900)
    base = _pipe(img, None).run(batches)
    for radius in (6, 2):
        pipe = _pipe(img, radius)
        out = pipe.run(batches)
        for b0, b1 in zip(base, out):
            for r0, r1 in zip(b0, b1):
                assert np.array_equal(r0["R"], r1["R"]) and np.array_equal(r0["t"], r1["t"])
                for k in ("best_cost", "initial_cost", "n_evals", "n_steps", "best_num_inliers", "status",
                          "texel_gathers"):
                    assert r0[k] == r1[k] or (k.endswith("cost") and np.isnan(r0[k]) and np.isnan(r1[k])), k
                assert r1["status"] & _lib.STATUS_WINDOW == 0
        if radius == 2:
            assert pipe.refills > 0  # the refill path ran
        print(init, radius, "refills", pipe.refills)


def test_window_miss_stops_the_problem_with_its_status():
    """A radius-2 window around the easy start: the LM reports FMPNP_STATUS_WINDOW for a query
    whose points move more than one texel (the pipeline's refill input)."""
    batches, img = _queries("easy", 1, 8, 950)
    pipe = _pipe(img, 2)
    batch, keep, err = pipe._prepare(batches[0], 0)
    torch.cuda.synchronize()  # the prep stream's descriptor upload, packs and gathers are done
    batch.launch(_lib.stream_ptr(DEV))
    res = batch.results()
    flagged = [r for r in res if r["status"] & _lib.STATUS_WINDOW]
    assert flagged, [r["status"] for r in res]
    base = _pipe(img, None).run(batches)[0]
    # unflagged queries are already the full pack's results
    for r, b in zip(res, base):
        if not r["status"] & _lib.STATUS_WINDOW:
            assert np.array_equal(r["R"], b["R"]) and r["best_cost"] == b["best_cost"]


def test_pipeline_channel_levels_equal_level_by_level_runs():
    """RefinePipeline(levels=...) (multilevel_optimization's channel pyramid, model.py:178-213,
    poses chained on the device) equals running each level as its own pipeline pass, the next
    level's initial pose taken from the previous level's results on the host."""
    levels = [(32, 64), (8, 32), (0, 8)]
    batches, img = synth.pipeline_queries(2, 5, N=128, C=64, Hf=48, Wf=64, device=DEV, seed0=1300)
    kw = dict(n_iters=20, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01, ratio_threshold=None)
    chained = RefinePipeline(img, storage=torch.float32, depth=2, levels=levels, model_kwargs=kw).run(batches)
    cur = batches
    for lv in levels:
        out = RefinePipeline(img, storage=torch.float32, depth=2, levels=[lv], model_kwargs=kw).run(cur)
        nxt = []
        for qs, rs in zip(cur, out):
            row = []
            for (a, b, p, k), r in zip(qs, rs):
                T = np.eye(4)
                T[:3, :3], T[:3, 3] = r["R"], r["t"]
                row.append((a, b, p._replace(matrix=T), k))
            nxt.append(row)
        cur = nxt
    for b0, b1 in zip(chained, out):
        for r0, r1 in zip(b0, b1):
            assert np.array_equal(r0["R"], r1["R"]) and np.array_equal(r0["t"], r1["t"])
            assert r0["best_cost"] == r1["best_cost"] and r0["n_evals"] == r1["n_evals"]
    with pytest.raises(ValueError):
        RefinePipeline(img, storage=torch.float32, levels=levels, window=5, model_kwargs=kw)
