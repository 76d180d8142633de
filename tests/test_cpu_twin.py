"""The CPU twin fmpnp_refine_batch_cpu (include/fmpnp.h) against the reference's
golden vectors and the oracle -- CPU only, no device.

Tolerances: fp64 texel storage reproduces the reference's trajectory (identical accept/reject
sequence and per-evaluation support counts, costs to 1e-10 relative, poses to 1e-9), as the
GPU path does (tests/test_gpu_parity.py); fp32 storage at the cfg2 shape within 1e-6 of the oracle."""
import math

import numpy as np
import pytest

import oracle.oracle as orc
from golden_io import FORWARD_CASES, case, maps64

from fmpnp import _lib, cpu, refine as rf

LOSS = {"squared": _lib.SQUARED, "huber": _lib.HUBER, "cauchy": _lib.CAUCHY, "geman_mcclure": _lib.GEMAN_MCCLURE,
        "barron": _lib.BARRON}


def accepts(costs):
    acc, prev = [], costs[0]
    for c in costs[1:]:
        a = not (c > prev)
        acc.append(a)
        if a:
            prev = c
    return acc


def run_case(name, dtype=np.float64, layout="fgrad", mode=_lib.MODE_FORWARD):
    inp, meta, gold = case(name)
    f, gx, gy = maps64(inp, orc.sobel)
    feats = cpu.pack_host(f, gx, gy, dtype) if layout == "fgrad" else cpu.pack_host(f, dtype=dtype, layout="f")
    prob = cpu.problem_host(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                            inp["R0"], inp["t0"])
    opts = rf.make_options(meta["n_iters"], meta["lambda0"], LOSS[meta["loss"]], meta.get("barron_alpha") or 0.0,
                           meta.get("ratio_threshold"), mode=mode)
    (res,), (tr,) = cpu.refine_cpu([prob], opts, trace=True, n_threads=1)
    return inp, meta, gold, res, tr


@pytest.mark.parametrize("name", FORWARD_CASES)
def test_twin_fp64_matches_reference(name):
    inp, meta, gold, res, tr = run_case(name)
    assert res["n_steps"] == int(gold["rec_n"])
    if "track_costs" in gold:
        gc = gold["track_costs"]
        assert len(tr["cost"]) == len(gc)
        np.testing.assert_allclose(tr["cost"], gc, rtol=1e-10, atol=0)
        assert list(tr["accepted"][1:]) == accepts(list(gc))
        np.testing.assert_array_equal(tr["n_supported"], gold["track_npts"])
        np.testing.assert_allclose(tr["R"], gold["track_R"], atol=1e-9)
        np.testing.assert_allclose(tr["t"], gold["track_t"], atol=1e-9)
        m = min(len(gc), int(gold["rec_n"]))
        np.testing.assert_array_equal(tr["lam"][1:m], gold["rec_lam"][1:m])
        np.testing.assert_array_equal(tr["lr"][1:m], gold["rec_lr"][1:m])
    np.testing.assert_allclose(res["R"], gold["out_R"], atol=1e-9)
    np.testing.assert_allclose(res["t"], gold["out_t"], atol=1e-9)
    assert res["has_best"] == bool(gold["has_best_cost_"])
    if res["has_best"]:
        assert res["best_cost"] == pytest.approx(float(gold["best_cost_"]), rel=1e-10)
        assert res["best_num_inliers"] == int(gold["best_num_inliers_"])
        assert res["initial_cost"] == pytest.approx(float(gold["initial_cost_"]), rel=1e-10)


def test_twin_kat_toy6():
    """FeatureBA_ToyExample.ipynb:477-478."""
    *_, res, tr = run_case("kat_toy6")
    assert tr["cost"][0] == pytest.approx(27497.41105769231, rel=1e-13)
    assert tr["cost"][-1] == pytest.approx(276.125, rel=1e-13)
    assert len(tr["cost"]) == 51


def test_twin_early_exits():
    *_, res, _ = run_case("no_support_init")
    assert res["status"] == _lib.STATUS_NO_SUPPORT and not res["has_best"] and res["n_evals"] == 0
    *_, res, _ = run_case("no_support_trial")
    assert res["status"] == _lib.STATUS_NO_SUPPORT_TRIAL


def test_twin_compute_cost_matches_golden():
    """FMPNP_MODE_COMPUTE_COST (model.py:216-243) against the reference's compute_cost golden: at the
    initial pose, the identity and a pose with no supported point (the reference returns None: status
    NO_SUPPORT), with and without the ratio test."""
    inp, meta, gold = case("compute_cost")
    f, gx, gy = maps64(inp, orc.sobel)
    feats = cpu.pack_host(f, gx, gy, np.float64)
    poses = {"init": (inp["R0"], inp["t0"]), "ident": (np.eye(3), np.zeros(3)),
             "away": (np.eye(3), np.array([500.0, 0.0, 0.0]))}
    for thr in (None, 0.8):
        for tag, (R, t) in poses.items():
            prob = cpu.problem_host(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                                    R, t)
            (res,), _ = cpu.refine_cpu([prob], rf.make_options(0, ratio_threshold=thr, mode=_lib.MODE_COMPUTE_COST))
            g = float(gold[f"cost_{tag}_{thr}"])
            if tag == "away":
                assert res["status"] == _lib.STATUS_NO_SUPPORT and math.isnan(res["initial_cost"])
            elif math.isnan(g):
                assert math.isnan(res["initial_cost"])
            else:
                assert res["initial_cost"] == pytest.approx(g, rel=1e-12)


@pytest.mark.parametrize("name", ["gm_c16", "ratio08_gm", "cauchy_c16"])
def test_twin_layout_f_equals_fgrad_fp64_sobel(name):
    """FMPNP_LAYOUT_F (the twin forms the fp64 Sobel of the fp32 map itself) against the fgrad layout
    with the oracle's fp64 gradients: the same sums, so the same trajectory to rounding."""
    inp, meta, gold = case(name)
    if "fmap32" not in inp:
        pytest.skip("fp64-only case")
    *_, a, ta = run_case(name, np.float32, "f")
    *_, b, tb = run_case(name, np.float64, "fgrad")
    np.testing.assert_array_equal(ta["n_supported"], tb["n_supported"])
    np.testing.assert_allclose(ta["cost"], tb["cost"], rtol=1e-9)
    np.testing.assert_allclose(a["R"], b["R"], atol=1e-9)


def test_twin_cfg2_fp32_against_oracle():
    """configs[1]'s shape (N=512, C=256, 240x320, GM, 50 iterations) from fp32 packed maps, against
    the oracle on the same map: identical support counts and accept sequence, costs to 1e-6."""
    from fmpnp import synth
    inp = synth.problem_inputs(512, 256, 240, 320, seed=3, device="cpu")
    fm = inp["fmap"].double().numpy()
    gx, gy = orc.sobel(fm)
    p = orc.make_problem(inp["pts3d"], inp["fref"].double().numpy(), fm, gx, gy, inp["K"], inp["im_width"],
                         inp["im_height"], inp["R0"], inp["t0"])
    ores, otr = orc.forward(p, orc.make_options(50, 0.01, "geman_mcclure"), trace_cap=51)
    feats = cpu.pack_host(inp["fmap"].numpy(), gx.astype(np.float32), gy.astype(np.float32), np.float32)
    prob = cpu.problem_host(feats, inp["fref"].numpy(), inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                            inp["R0"], inp["t0"])
    (res,), (tr,) = cpu.refine_cpu([prob], rf.make_options(50, 0.01, _lib.GEMAN_MCCLURE), trace=True)
    np.testing.assert_array_equal(tr["n_supported"], otr["n_supported"])
    np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-6)
    assert res["n_evals"] == ores["n_evals"] and res["n_steps"] == ores["n_steps"]
    assert np.linalg.norm(res["t"] - ores["t"]) < 1e-4
    assert 0 < res["texel_gathers"] < 51 * 512  # (memoised: a point re-reads its texel only when it changes)


def test_twin_batch_threads_equal_serial():
    """Problems are independent: a batch over several host threads equals one thread, bit for bit."""
    probs = []
    for name in ("gm_c16", "cauchy_c16", "ratio08_gm", "huber_c16"):
        inp, meta, gold = case(name)
        f, gx, gy = maps64(inp, orc.sobel)
        probs.append(cpu.problem_host(cpu.pack_host(f, gx, gy, np.float64), inp["fref"], inp["pts3d"], inp["K"],
                                      inp["im_width"], inp["im_height"], inp["R0"], inp["t0"]))
    opts = rf.make_options(30, 0.01, _lib.GEMAN_MCCLURE)
    a, _ = cpu.refine_cpu(probs, opts, n_threads=1)
    b, _ = cpu.refine_cpu(probs, opts, n_threads=4)
    for x, y in zip(a, b):
        assert np.array_equal(x["R"], y["R"]) and np.array_equal(x["t"], y["t"]) and x["best_cost"] == y["best_cost"]


def test_twin_rejects_bad_arguments():
    inp, meta, gold = case("gm_c16")
    f, gx, gy = maps64(inp, orc.sobel)
    prob = cpu.problem_host(cpu.pack_host(f, gx, gy, np.float64), inp["fref"], inp["pts3d"], inp["K"],
                            inp["im_width"], inp["im_height"], inp["R0"], inp["t0"])
    with pytest.raises(_lib.FmpnpError):
        cpu.refine_cpu([prob], rf.make_options(5, sampling="bilinear"))
    o = rf.make_options(5)
    o.loss = 9
    with pytest.raises(_lib.FmpnpError):
        cpu.refine_cpu([prob], o)
