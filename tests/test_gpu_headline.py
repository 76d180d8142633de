"""Full-length parity of the headline kernel on the BASELINE shapes (needs an MI355X).

The bench's kernel variant -- fp32 texels, packed f/gx/gy ("fgrad") layout, memoised
gathers, Geman-McClure -- run for the reference's full iteration count
(featurePnP/model.gin:5, n_iters = 50; the loop of featurePnP/model.py:300-486) at the
configs[1] shape (N=512, C=256, 240x320), and as configs[2]'s per-GPU work: a batch of
16 distinct-map queries in ONE launch, seeded like bench.py (seed = global query index).
Each query is checked against its own run of the oracle (oracle/, the C restatement of
the reference loop, fp64 CHW maps with the fp64 Sobel of the same fp32 hypercolumn).

Tolerance (north star, BASELINE.json): final pose within 1e-4 rad / 1e-4 m after the
same iteration count; the per-evaluation support counts (model.py:311,436) identical, so
the accept/reject trajectory has the same length; costs within 1e-6 relative (fp32 texels
and fp32-rounded packed gradients against the oracle's fp64 ones).
"""
import math
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

import oracle.oracle as orc

pytestmark = pytest.mark.gpu

from fmpnp import _lib, refine as rf, synth  # noqa: E402  (no skip: a missing HIP library must fail)

DEV = "cuda:0"
ITERS = 50
LOSS = {"geman_mcclure": _lib.GEMAN_MCCLURE, "cauchy": _lib.CAUCHY}


def rot_angle(Ra, Rb):
    c = (np.trace(np.asarray(Ra).T @ np.asarray(Rb)) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


def oracle_run(host_inp, n_iters=ITERS, loss="geman_mcclure", ratio=None):
    """The oracle on one query's host copy (fmap fp64 = the fp32 map, exact; fp64 Sobel)."""
    fm = host_inp["fmap"]
    gx, gy = orc.sobel(fm)
    p = orc.make_problem(host_inp["pts3d"], host_inp["fref"], fm, gx, gy, host_inp["K"], host_inp["im_width"],
                         host_inp["im_height"], host_inp["R0"], host_inp["t0"])
    return orc.forward(p, orc.make_options(n_iters, 0.01, loss, ratio), trace_cap=n_iters + 1)


def host_copy(inp):
    return dict(inp, fmap=inp["fmap"].double().cpu().numpy(), fref=inp["fref"].double().cpu().numpy())


def check(res, tr, ores, otr, what):
    assert res["status"] == 0, what
    assert rot_angle(res["R"], ores["R"]) < 1e-4, what
    assert np.linalg.norm(res["t"] - ores["t"]) < 1e-4, what
    assert res["n_evals"] == ores["n_evals"] and res["n_steps"] == ores["n_steps"], what
    if tr is not None:
        np.testing.assert_array_equal(tr["n_supported"], otr["n_supported"], err_msg=what)
        np.testing.assert_array_equal(tr["n_kept"], otr["n_kept"], err_msg=what)  # (the ratio test's kept set)
        np.testing.assert_allclose(tr["cost"], otr["cost"], rtol=1e-6, err_msg=what)
    assert res["best_num_inliers"] == ores["best_num_inliers"], what
    assert res["best_cost"] == pytest.approx(ores["best_cost"], rel=1e-6), what


def packed_problem(inp, layout="fgrad"):
    feats = rf.pack_features(inp["fmap"], storage=torch.float32, device=DEV, layout=layout)
    return rf.make_problem(feats, inp["fref"], inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                           inp["R0"], inp["t0"])


@pytest.mark.parametrize("init,ratio", [("easy", None), ("hard", None), ("hard", 0.8), ("easy", 0.8)])
def test_cfg2_single_query_50_iters(init, ratio):
    """configs[1]: one query, the bench's kernel variant, 50 iterations, vs the oracle.  'hard'
    is the golden vectors' perturbation (several texels of motion); 0.8 the ratio test of
    input_configs/full_robotcar_08.gin:40."""
    inp = synth.problem_inputs(512, 256, 240, 320, seed=3, device=DEV, init=init)
    ores, otr = oracle_run(host_copy(inp), ratio=ratio)
    prob = packed_problem(inp)
    (res,), (tr,) = rf.refine([prob], rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, ratio_threshold=ratio,
                                                      dtype=_lib.F32), trace=True)
    check(res, tr, ores, otr, f"{init} ratio={ratio}")


def test_cfg2_batch_of_16_distinct_maps_in_one_launch():
    """configs[2]'s per-GPU work in miniature: 16 cfg2 queries with distinct maps (seeded by
    global query index, as bench.py), ONE launch of the bench's AsyncBatch path, every
    query against its own oracle run; the traced synchronous launch of the same batch
    gives the same poses bit for bit and the per-evaluation support counts."""
    B = 16
    inps = [synth.problem_inputs(512, 256, 240, 320, seed=q, device=DEV) for q in range(B)]
    hosts = [host_copy(i) for i in inps]
    probs = [packed_problem(i) for i in inps]
    del inps
    opts = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
    ab = rf.AsyncBatch(probs, opts)
    ab.launch()
    res_async = ab.results()
    assert _lib.last_launch()["grid"] >= B
    res, trs = rf.refine(probs, opts, trace=True)
    with ThreadPoolExecutor(8) as ex:
        oracle = list(ex.map(oracle_run, hosts))
    for q in range(B):
        assert np.array_equal(res[q]["R"], res_async[q]["R"]) and np.array_equal(res[q]["t"], res_async[q]["t"])
        check(res[q], trs[q], *oracle[q], f"query {q}")


@pytest.mark.parametrize("layout", ["fgrad", "f"])
def test_cfg5_cauchy_50_iters(layout):
    """configs[4] (N=2048, C=512, 480x640, Cauchy, robotcar_inlier_GN.gin:39): the
    multi-round gather and a team of workgroups per problem, 50 iterations vs the oracle."""
    inp = synth.problem_inputs(2048, 512, 480, 640, seed=5, device=DEV)
    host = host_copy(inp)
    prob = packed_problem(inp, layout)
    del inp
    (res,), (tr,) = rf.refine([prob], rf.make_options(ITERS, 0.01, _lib.CAUCHY, dtype=_lib.F32), trace=True)
    assert _lib.last_launch()["wgs_per_problem"] >= 2
    del prob
    ores, otr = oracle_run(host, loss="cauchy")
    check(res, tr, ores, otr, f"cfg5 {layout}")


def test_cfg2_layout_f_50_iters():
    """The f-only layout (the streamed pipeline's default): the LM gather forms the fp64
    Sobel of the fp32 map itself, so it sees the oracle's gradients exactly."""
    inp = synth.problem_inputs(512, 256, 240, 320, seed=11, device=DEV, init="hard")
    ores, otr = oracle_run(host_copy(inp))
    prob = packed_problem(inp, "f")
    (res,), (tr,) = rf.refine([prob], rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32), trace=True)
    check(res, tr, ores, otr, "layout f")


@pytest.mark.parametrize("layout,init,ratio,wgs", [("fgrad", "easy", None, 0), ("fgrad", "hard", 0.8, 0),
                                                   ("f", "hard", None, 0), ("fgrad", "hard", None, 3)])
def test_speculative_gathers_change_nothing(layout, init, ratio, wgs):
    """The speculative next-texel gathers (fmpnp_lm_impl.h spec_pass) only move where a
    record's sums come from: poses, costs, support counts and the LM schedule are
    bit-identical with speculation on, off, and with memoisation off."""
    inp = synth.problem_inputs(512, 256, 240, 320, seed=21, device=DEV, init=init)
    prob = packed_problem(inp, layout)
    runs = []
    for memo, spec in ((True, True), (True, False), (False, False)):
        o = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, ratio_threshold=ratio, dtype=_lib.F32,
                            wgs_per_problem=wgs, memoize=memo, speculate=spec)
        (res,), (tr,) = rf.refine([prob], o, trace=True)
        runs.append((res, tr))
    (a, ta), (b, tb), (c, tc) = runs
    for r, t in ((b, tb), (c, tc)):
        assert np.array_equal(a["R"], r["R"]) and np.array_equal(a["t"], r["t"])
        assert a["best_cost"] == r["best_cost"] and a["n_evals"] == r["n_evals"]
        np.testing.assert_array_equal(ta["cost"], t["cost"])
        np.testing.assert_array_equal(ta["n_supported"], t["n_supported"])
    # speculation reads more texels in total, but the evaluations themselves gather fewer
    assert c["texel_gathers"] >= b["texel_gathers"]


@pytest.mark.parametrize("w0,cap", [("0", "4"), ("1", "64"), ("3", "2"), ("4", "0"), ("4", "2"), ("4", "4"), ("8", "4")])
def test_speculation_settings_change_nothing(w0, cap, monkeypatch):
    """Which waves speculate (FMPNP_SPEC_W0: the default 3 adds wave 3, idle in the tail, to the
    later wave of each SIMD; 0 adds wave 0's held pair; 8 none) and how many texels each gathers per evaluation
    (FMPNP_SPEC_CAP; a withdrawn prediction is gathered on demand) only move where sums come
    from: bit-identical to the run without speculation."""
    if not _lib.spec_build():
        pytest.skip("library built without speculation")
    inp = synth.problem_inputs(512, 256, 240, 320, seed=23, device=DEV, init="hard")
    prob = packed_problem(inp, "fgrad")
    o = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, speculate=False)
    (base,), (tb,) = rf.refine([prob], o, trace=True)
    monkeypatch.setenv("FMPNP_SPEC_W0", w0)
    monkeypatch.setenv("FMPNP_SPEC_CAP", cap)
    o = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32, speculate=True)
    (r,), (t,) = rf.refine([prob], o, trace=True)
    assert np.array_equal(base["R"], r["R"]) and np.array_equal(base["t"], r["t"])
    assert base["best_cost"] == r["best_cost"] and base["n_evals"] == r["n_evals"]
    np.testing.assert_array_equal(tb["cost"], t["cost"])
    np.testing.assert_array_equal(tb["n_supported"], t["n_supported"])
    np.testing.assert_array_equal(tb["lam"], t["lam"])


@pytest.mark.parametrize("B,init,ratio,C,spec", [(1, "easy", None, 256, True), (1, "hard", 0.8, 256, True),
                                                  (4, "hard", None, 256, True), (16, "easy", None, 256, True),
                                                  (2, "hard", None, 512, True), (1, "easy", None, 256, False)])
def test_first_evaluation_helpers_change_nothing(B, init, ratio, C, spec, monkeypatch):
    """Small batches: helper workgroups gather the first evaluation's records of each problem's
    64-point blocks on otherwise idle CUs (fmpnp_lm_impl.h helper_run).  Same gather code at the
    same pose, so poses, costs, support counts, the LM schedule and the gather counts are
    bit-identical to the run without helpers."""
    H, W = (240, 320) if C == 256 else (120, 160)
    probs = [packed_problem(synth.problem_inputs(512, C, H, W, seed=40 + q, device=DEV, init=init), "fgrad")
             for q in range(B)]
    o = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, ratio_threshold=ratio, dtype=_lib.F32, speculate=spec)
    monkeypatch.setenv("FMPNP_HELPERS", "0")
    base, tb = rf.refine(probs, o, trace=True)
    assert _lib.last_launch()["grid"] == B
    monkeypatch.setenv("FMPNP_HELPERS", "1")
    res, tr = rf.refine(probs, o, trace=True)
    assert _lib.last_launch()["grid"] > B  # the helpers ran
    for q in range(B):
        a, r = base[q], res[q]
        assert np.array_equal(a["R"], r["R"]) and np.array_equal(a["t"], r["t"]), q
        assert a["best_cost"] == r["best_cost"] and a["n_evals"] == r["n_evals"] and a["status"] == r["status"]
        assert a["texel_gathers"] == r["texel_gathers"]
        np.testing.assert_array_equal(tb[q]["cost"], tr[q]["cost"])
        np.testing.assert_array_equal(tb[q]["n_supported"], tr[q]["n_supported"])
        np.testing.assert_array_equal(tb[q]["lam"], tr[q]["lam"])


def test_first_evaluation_helpers_fp64_storage(monkeypatch):
    """The helpers' hand-off with fp64 texels (VAR_GM_H, the non-speculating variant at C = 256
    fp64): bit-identical to the run without helpers."""
    inp = synth.problem_inputs(512, 256, 240, 320, seed=47, device=DEV, init="hard")
    feats = rf.pack_features(inp["fmap"].double(), storage=torch.float64, device=DEV)
    prob = rf.make_problem(feats, inp["fref"].double(), inp["pts3d"], inp["K"], inp["im_width"], inp["im_height"],
                           inp["R0"], inp["t0"])
    o = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F64)
    monkeypatch.setenv("FMPNP_HELPERS", "0")
    (base,), (tb,) = rf.refine([prob], o, trace=True)
    monkeypatch.setenv("FMPNP_HELPERS", "1")
    (res,), (tr,) = rf.refine([prob], o, trace=True)
    assert _lib.last_launch()["grid"] > 1
    assert np.array_equal(base["R"], res["R"]) and np.array_equal(base["t"], res["t"])
    assert base["best_cost"] == res["best_cost"] and base["texel_gathers"] == res["texel_gathers"]
    np.testing.assert_array_equal(tb["cost"], tr["cost"])
    np.testing.assert_array_equal(tb["n_supported"], tr["n_supported"])


# ---------------------------------------------------------------------------
# The EXACT launches bench.py times, at the launch shapes it times them (configs[2]'s per-GPU
# share of 128 queries; the fixed total of 1024 on one GPU takes the same two-workgroups-per-CU
# build as B = 512): the plan of each launch is asserted (grid, build, variant, no helpers), and a
# spread subset of >= 32 queries is compared with its own oracle run, trace included.
# ---------------------------------------------------------------------------
def _bench_batch(B):
    """bench.py's setup: query q = synth.problem_inputs(seed=q), packed fp32 f/gx/gy."""
    probs = []
    for q in range(B):
        inp = synth.problem_inputs(512, 256, 240, 320, seed=q, device=DEV)
        probs.append(packed_problem(inp))
        del inp
    return probs


def _oracle_subset(qs, ratio):
    def one(q):
        return oracle_run(host_copy(synth.problem_inputs(512, 256, 240, 320, seed=q, device=DEV)), ratio=ratio)
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(one, qs))


@pytest.mark.parametrize("B,ratio,build,variant", [(128, None, "latency", "GM_SPEC_512"),
                                                   (128, 0.8, "latency", "GM_SPEC_512"),
                                                   (512, None, "throughput", "GM"),
                                                   (512, 0.8, "throughput", "GM")])
def test_bench_launch_against_oracle(B, ratio, build, variant):
    """The headline launch (B = 128: lm_kernel<float, latency, !team, ratio, VAR_GM_SPEC_512>, grid 128,
    no first-evaluation helpers), its ratio-test form (input_configs/full_robotcar_08.gin:40), and
    the throughput build of B >= 512 (the fixed_total_1024 leg), each as bench.py launches it
    (AsyncBatch), against the oracle (featurePnP/model.py:300-486, n_iters = 50 of model.gin:5)."""
    probs = _bench_batch(B)
    opts = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, ratio_threshold=ratio, dtype=_lib.F32)
    ab = rf.AsyncBatch(probs, opts)
    ab.launch()
    res_async = ab.results()
    info = _lib.last_launch()
    assert (info["grid"], info["wgs_per_problem"], info["helpers"]) == (B, 1, 0), info
    assert (info["build_name"], info["variant_name"], info["ratio"], info["dtype_name"]) == \
        (build, variant, int(ratio is not None), "f32"), info
    # the traced synchronous launch of the same batch: same plan, same poses bit for bit
    res, trs = rf.refine(probs, opts, trace=True)
    info2 = _lib.last_launch()
    assert {k: info2[k] for k in ("grid", "build", "variant", "helpers", "team")} == \
        {k: info[k] for k in ("grid", "build", "variant", "helpers", "team")}
    for q in range(B):
        assert np.array_equal(res[q]["R"], res_async[q]["R"]) and np.array_equal(res[q]["t"], res_async[q]["t"]), q
        assert res[q]["n_evals"] == res_async[q]["n_evals"] and res[q]["status"] == res_async[q]["status"] == 0
    del probs
    qs = list(range(0, B, B // 32))  # 32 queries spread over the batch
    for q, (ores, otr) in zip(qs, _oracle_subset(qs, ratio)):
        check(res[q], trs[q], ores, otr, f"B={B} ratio={ratio} query {q}")


def test_helpers_on_a_reused_workspace(monkeypatch):
    """the first-evaluation helpers' records live in the launch workspace.  Batch A
    then batch B (other maps, other points) on ONE reused workspace with helpers on must give B's
    helpers-off results bit for bit -- no record of A can be taken for B's (launch-unique tags,
    release/acquire hand-off, texel check)."""
    mk = lambda seeds: [packed_problem(synth.problem_inputs(512, 256, 240, 320, seed=s, device=DEV, init="hard"))
                        for s in seeds]
    pa, pb = mk(range(60, 64)), mk(range(70, 74))
    o = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
    monkeypatch.setenv("FMPNP_HELPERS", "0")
    base, tb = rf.refine(pb, o, trace=True)
    monkeypatch.setenv("FMPNP_HELPERS", "1")
    ab_a, ab_b = rf.AsyncBatch(pa, o), rf.AsyncBatch(pb, o)
    ab_b.d_ws = ab_a.d_ws  # one workspace for both batches
    ab_b.ws_bytes = ab_a.ws_bytes
    for _ in range(3):
        ab_a.launch()
        ab_b.launch()
        assert _lib.last_launch()["helpers"] > 0
        got = ab_b.results()
        for q in range(len(pb)):
            assert np.array_equal(got[q]["R"], base[q]["R"]) and np.array_equal(got[q]["t"], base[q]["t"]), q
            assert got[q]["best_cost"] == base[q]["best_cost"] and got[q]["n_evals"] == base[q]["n_evals"]
            assert got[q]["texel_gathers"] == base[q]["texel_gathers"] and got[q]["status"] == 0


def test_helpers_that_never_publish_change_nothing(monkeypatch):
    """A helper that never publishes (FMPNP_DBG bit 3: the state a helper kept from being resident
    leaves): every main workgroup waits its bounded 0.2 s per block, gathers the block itself and
    reports FMPNP_STATUS_HELPER_WAIT; poses, costs and the schedule are bit-identical."""
    prob = packed_problem(synth.problem_inputs(512, 256, 240, 320, seed=81, device=DEV, init="hard"))
    o = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, dtype=_lib.F32)
    monkeypatch.setenv("FMPNP_HELPERS", "0")
    (base,), (tb,) = rf.refine([prob], o, trace=True)
    monkeypatch.setenv("FMPNP_HELPERS", "1")
    monkeypatch.setenv("FMPNP_DBG", "8")
    (res,), (tr,) = rf.refine([prob], o, trace=True)
    assert _lib.last_launch()["helpers"] > 0
    assert res["status"] == _lib.STATUS_HELPER_WAIT and base["status"] == 0
    assert np.array_equal(base["R"], res["R"]) and np.array_equal(base["t"], res["t"])
    assert base["best_cost"] == res["best_cost"] and base["texel_gathers"] == res["texel_gathers"]
    np.testing.assert_array_equal(tb["cost"], tr["cost"])
    np.testing.assert_array_equal(tb["n_supported"], tr["n_supported"])


@pytest.mark.parametrize("B,init,ratio", [(128, "easy", 0.8), (128, "hard", 0.8), (16, "easy", 0.5), (1, "hard", 0.8),
                                          (512, "easy", 0.8)])
def test_ratio_guess_changes_nothing(B, init, ratio, monkeypatch):
    """The ratio test with a guessed limit (fmpnp_lm_impl.h ratio_guess_check: block partials formed
    in pass 1 with the previous evaluation's limit, re-formed only when the true limit crosses a
    point) against the same kernel forced to re-form every evaluation (FMPNP_DBG bit 5, the
    two-pass partials): poses, costs, support and kept counts bit-identical, and the guess right in
    most evaluations (FMPNP_DBG bit 6 counts the re-forms)."""
    probs = [packed_problem(synth.problem_inputs(512, 256, 240, 320, seed=q, device=DEV, init=init))
             for q in range(B)]
    o = rf.make_options(ITERS, 0.01, _lib.GEMAN_MCCLURE, ratio_threshold=ratio, dtype=_lib.F32)
    monkeypatch.setenv("FMPNP_DBG", "96")  # every evaluation re-formed, counted
    base, tb = rf.refine(probs, o, trace=True)
    assert _lib.last_launch()["ratio"] == 1  # (B = 512: the throughput build, two blocks per wave)
    monkeypatch.setenv("FMPNP_DBG", "64")  # the guess, re-forms counted
    res, tr = rf.refine(probs, o, trace=True)
    redo = sum(r["texel_gathers"] >> 32 for r in res)  # (re-formed 64-point blocks)
    evals = sum(r["n_evals"] for r in res)
    for q in range(B):
        assert np.array_equal(res[q]["R"], base[q]["R"]) and np.array_equal(res[q]["t"], base[q]["t"]), q
        assert res[q]["best_cost"] == base[q]["best_cost"] and res[q]["n_evals"] == base[q]["n_evals"], q
        np.testing.assert_array_equal(tr[q]["cost"], tb[q]["cost"])
        np.testing.assert_array_equal(tr[q]["n_supported"], tb[q]["n_supported"])
        np.testing.assert_array_equal(tr[q]["n_kept"], tb[q]["n_kept"])
        assert (res[q]["texel_gathers"] & 0xFFFFFFFF) == (base[q]["texel_gathers"] & 0xFFFFFFFF)
    assert sum(r["texel_gathers"] >> 32 for r in base) == 8 * evals  # (forced: every block of every evaluation)
    print(f"B={B} {init} ratio {ratio}: re-formed {redo} of {8 * evals} blocks")
    assert redo < 4 * evals


@pytest.mark.parametrize("B", [1, 128])
def test_cfg0_toy_shape_against_oracle(B):
    """configs[0]'s stated shape (featurePnP/toy_example: N=64 points, C=3, 120x160, squared loss,
    20 GN iterations), batch 1 and 128 distinct maps in one launch, each against its own oracle
    run (the toy-6 KAT covers the reference's own toy data, tests/test_gpu_parity.py)."""
    inps = [synth.problem_inputs(64, 3, 120, 160, seed=300 + q, device=DEV) for q in range(B)]
    hosts = [host_copy(i) for i in inps]
    probs = [packed_problem(i) for i in inps]
    del inps
    res, trs = rf.refine(probs, rf.make_options(20, 0.01, _lib.SQUARED, dtype=_lib.F32), trace=True)
    with ThreadPoolExecutor(8) as ex:
        oracle = list(ex.map(lambda h: oracle_run(h, n_iters=20, loss="squared"), hosts))
    for q in range(B):
        check(res[q], trs[q], *oracle[q], f"toy query {q}")
