"""Edge cases of the HIP refiner (all checked against the oracle or against bit-level
invariants the design promises):
  * memoisation off re-reads every texel and is bit-identical to the default;
  * N = 0 and N = 1 problems (early exit / a single point);
  * the per-evaluation trace does not depend on the workgroups per problem;
  * channel slices with unaligned bounds (scalar gather path) follow the oracle;
  * a batch mixing problem sizes that need different team sizes matches single launches.
"""
import math

import numpy as np
import pytest
import torch

import oracle.oracle as orc
from golden_io import case, maps64

pytestmark = pytest.mark.gpu

from fmpnp import _lib, refine as rf, synth  # noqa: E402

DEV = "cuda:0"


def packed_case(name, storage=torch.float64):
    inp, meta, _ = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    feats = rf.pack_features(torch.from_numpy(f).to(storage), torch.from_numpy(gx).to(storage),
                             torch.from_numpy(gy).to(storage), storage=storage, device=DEV)
    return inp, meta, f, gx, gy, feats


def test_memoisation_off_is_bit_identical():
    inputs = synth.problem_inputs(512, 256, 240, 320, seed=21, device=DEV)
    feats = rf.pack_features(inputs["fmap"], storage=torch.float32, device=DEV)
    prob = rf.make_problem(feats, inputs["fref"], inputs["pts3d"], inputs["K"], inputs["im_width"],
                           inputs["im_height"], inputs["R0"], inputs["t0"])
    (a,), (ta,) = rf.refine([prob], rf.make_options(30, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32), trace=True)
    (b,), (tb,) = rf.refine([prob], rf.make_options(30, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, memoize=False),
                            trace=True)
    assert np.array_equal(a["R"], b["R"]) and np.array_equal(a["t"], b["t"])
    assert np.array_equal(ta["cost"], tb["cost"])
    assert b["texel_gathers"] > 5 * a["texel_gathers"]  # memo off re-reads every supported point


@pytest.mark.parametrize("n", [0, 1])
def test_tiny_problems(n):
    inp, meta, f, gx, gy, feats = packed_case("gm_c16")
    pts, fref = inp["pts3d"][:n], inp["fref"][:n]
    prob = rf.make_problem(feats, torch.from_numpy(fref.reshape(n, -1) if n else np.zeros((0, fref.shape[1]))),
                           pts.reshape(n, 3), inp["K"], inp["im_width"], inp["im_height"], inp["R0"], inp["t0"])
    (res,), _ = rf.refine([prob], rf.make_options(10, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F64))
    if n == 0:
        assert res["status"] == _lib.STATUS_NO_SUPPORT and not res["has_best"]
        np.testing.assert_array_equal(res["R"], np.asarray(inp["R0"]).reshape(3, 3))
        return
    p = orc.make_problem(pts, fref, f, gx, gy, inp["K"], inp["im_width"], inp["im_height"], inp["R0"], inp["t0"])
    ores, _ = orc.forward(p, orc.make_options(10, 0.01, "geman_mcclure"))
    np.testing.assert_allclose(res["R"], ores["R"], atol=1e-9)
    np.testing.assert_allclose(res["t"], ores["t"], atol=1e-9)


def test_trace_independent_of_workgroups_per_problem():
    inp, meta, f, gx, gy, feats = packed_case("ratio08_gm")
    prob = rf.make_problem(feats, torch.from_numpy(inp["fref"]), inp["pts3d"], inp["K"], inp["im_width"],
                           inp["im_height"], inp["R0"], inp["t0"])
    traces = []
    for g in (1, 2):
        opts = rf.make_options(meta["n_iters"], meta["lambda0"], _lib.GEMAN_MCCLURE, 0.0, meta["ratio_threshold"],
                               _lib.F64, wgs_per_problem=g)
        (_,), (tr,) = rf.refine([prob], opts, trace=True)
        traces.append(tr)
    for k in ("cost", "lam", "lr", "n_supported", "n_kept", "accepted", "R", "t"):
        assert np.array_equal(traces[0][k], traces[1][k]), k


@pytest.mark.parametrize("c_begin,c_end", [(1, 7), (3, 16), (5, 6)])
def test_unaligned_channel_slice_follows_oracle(c_begin, c_end):
    """c_begin / c_end not multiples of the 16-byte vector: the scalar gather path."""
    inp, meta, f, gx, gy, feats = packed_case("gm_c16")
    prob = rf.make_problem(feats, torch.from_numpy(inp["fref"]), inp["pts3d"], inp["K"], inp["im_width"],
                           inp["im_height"], inp["R0"], inp["t0"], c_begin, c_end)
    (res,), (tr,) = rf.refine([prob], rf.make_options(15, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F64), trace=True)
    p = orc.make_problem(inp["pts3d"], inp["fref"], f, gx, gy, inp["K"], inp["im_width"], inp["im_height"],
                         inp["R0"], inp["t0"], c_begin, c_end)
    ores, otr = orc.forward(p, orc.make_options(15, 0.01, "geman_mcclure"), 32)
    np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-10)
    np.testing.assert_allclose(res["R"], ores["R"], atol=1e-9)
    np.testing.assert_allclose(res["t"], ores["t"], atol=1e-9)


def test_mixed_sizes_in_one_batch_match_single_launches():
    """Problems of different N (1..3 blocks) and map sizes in one launch with teams of G = 2
    workgroups (requested: the planner keeps 512-point problems on one workgroup): every
    result equals its single-problem launch (planner's G = 1)."""
    probs = []
    for s, (n, c, h, w) in enumerate([(37, 8, 30, 40), (130, 16, 60, 80), (64, 12, 45, 50), (190, 4, 20, 30)]):
        inp = synth.problem_inputs(n, c, h, w, seed=40 + s, device=DEV)
        feats = rf.pack_features(inp["fmap"], storage=torch.float64, device=DEV)
        probs.append(rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                     inp["R0"], inp["t0"]))
    opts = rf.make_options(20, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F64)
    batch, _ = rf.refine(probs, rf.make_options(20, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F64, wgs_per_problem=2))
    assert _lib.last_launch()["wgs_per_problem"] == 2
    for p, rb in zip(probs, batch):
        (r1,), _ = rf.refine([p], opts)
        assert np.array_equal(r1["R"], rb["R"]) and np.array_equal(r1["t"], rb["t"])
        assert r1["best_cost"] == rb["best_cost"] or (math.isnan(r1["best_cost"]) and math.isnan(rb["best_cost"]))


def _bil_problem(inp, feats, n):
    pts, fref = inp["pts3d"][:n], inp["fref"][:n]
    return rf.make_problem(feats, torch.from_numpy(fref.reshape(n, -1) if n else np.zeros((0, fref.shape[1]))),
                           pts.reshape(n, 3), inp["K"], inp["im_width"], inp["im_height"], inp["R0"], inp["t0"])


def test_bilinear_memo_one_team_walks_mixed_sizes():
    """The bilinear cell memo keeps per-workgroup state (the dirty ballots, the memo columns)
    from one problem to the next: one team (max_teams = 1) walking problems of 0, 1, all and
    65 points -- the empty one right after a full one -- gives each problem's own results,
    equal to its single launch and, for the non-empty ones, to the oracle."""
    inp, meta, f, gx, gy, feats = packed_case("gm_c16")
    N = inp["pts3d"].shape[0]
    sizes = [N, 0, 1, N, 65 if N > 65 else N - 1]
    probs = [_bil_problem(inp, feats, n) for n in sizes]
    opts = dict(dtype=_lib.F64, sampling="bilinear")
    res, _ = rf.refine(probs, rf.make_options(12, 0.01, _lib.GEMAN_MCCLURE, max_teams=1, **opts))
    for n, p, r in zip(sizes, probs, res):
        (single,), _ = rf.refine([p], rf.make_options(12, 0.01, _lib.GEMAN_MCCLURE, **opts))
        assert np.array_equal(r["R"], single["R"]) and np.array_equal(r["t"], single["t"]), n
        assert r["status"] == single["status"], n
        if n == 0:
            assert r["status"] == _lib.STATUS_NO_SUPPORT
            continue
        op = orc.make_problem(inp["pts3d"][:n], inp["fref"][:n], f, gx, gy, inp["K"], inp["im_width"],
                              inp["im_height"], inp["R0"], inp["t0"])
        ores, _ = orc.forward(op, orc.make_options(12, 0.01, "geman_mcclure", sampling="bilinear"))
        np.testing.assert_allclose(r["R"], ores["R"], atol=1e-9)
        np.testing.assert_allclose(r["t"], ores["t"], atol=1e-9)


@pytest.mark.parametrize("span", [256, 384, 512, 640, 1024])
def test_vector_and_scalar_gathers_are_bit_identical(span):
    """The gather's 16-byte vector form (aligned channel slice) and its scalar form (a slice
    starting one channel into the 16-byte vector) accumulate every lane's channels in the same
    (round, element) order, so the same channel values give the same six sums -- in every regime
    of the vector form: one round pair (64 V = 256 fp32 channels), 64 V < C <= 128 V (384, 512),
    and the chunks of four rounds above it (640: a ragged last chunk; 1024: the RobotCar
    hypercolumn's [640:1664] slice).  Map B holds map A's channels shifted by three, so B's slice
    [1, 1 + span) (scalar path) has A's slice [4, 4 + span) (vector path) channel for channel."""
    N, H, W = 128, 24, 32
    inp = synth.problem_inputs(N, span + 8, H, W, seed=61, device=DEV, init="hard")
    fa, ra = inp["fmap"], inp["fref"]
    fb = torch.cat([fa[3:], torch.zeros_like(fa[:3])])
    rb = torch.cat([ra[:, 3:], torch.zeros_like(ra[:, :3])], 1)
    args = (inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"], inp["R0"], inp["t0"])
    pa = rf.make_problem(rf.pack_features(fa, storage=torch.float32, device=DEV), ra, *args, 4, 4 + span)
    pb = rf.make_problem(rf.pack_features(fb, storage=torch.float32, device=DEV), rb, *args, 1, 1 + span)
    opts = rf.make_options(25, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, wgs_per_problem=1)
    (a,), (ta,) = rf.refine([pa], opts, trace=True)
    (b,), (tb,) = rf.refine([pb], opts, trace=True)
    assert ta["n_supported"].min() > 0
    for k in ("cost", "n_supported", "accepted", "R", "t"):
        assert np.array_equal(ta[k], tb[k]), k
    assert np.array_equal(a["R"], b["R"]) and np.array_equal(a["t"], b["t"])
