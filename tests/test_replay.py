"""Cached-matches replay (the reference's --only_optimization path,
s2dhm/pose_prediction/sparse_to_dense_predictor.py:29-39, 192-231).

CPU: the reference's on-disk format (pickled entry dicts in cached_matches/*.npz, written
here by this test itself) reads back, converts to the pickle-free flat format and back, and
`prediction_from_entry` applies the inlier mask as :210-222 does.  GPU: one batched replay
launch over several cached queries reproduces the reference's own feature_pnp outputs for
the golden adapter case (tests/golden/adapter_square.npz, produced by the reference).
"""
import json
import os

import numpy as np
import pytest

from golden_io import load_npz

from fmpnp import replay as rp  # noqa: E402  (pure host code; no device needed to import)

# sparse_to_dense_predictor.py:102 columns as written by :285 (header line of the reference's
# results/results_s2dhm/robotcar/summary.csv)
REFERENCE_SUMMARY_HEADER = (";reference_image_origin;query_image_origin;num_initial_matches;num_final_matches;"
                            "initial_cost;final_cost;track_pickle_path")


def golden_entries(n_ok=4, n_fail=1):
    z = load_npz("adapter_square")
    N = z["in_points_3d"].shape[0]
    rng = np.random.default_rng(0)
    # two extra outlier rows that the inlier mask removes (:211-213)
    ref2d = np.concatenate([z["in_reference_inliers"], rng.uniform(0, 190, (2, 2))])
    q2d = np.concatenate([rng.uniform(0, 190, (N, 2)), rng.uniform(0, 190, (2, 2))])
    p3d = np.concatenate([z["in_points_3d"].reshape(N, 3), rng.normal(size=(2, 3))]).reshape(-1, 1, 3)
    mask = np.ones(N + 2, bool)
    mask[-2:] = False
    entries = {}
    for i in range(n_ok + n_fail):
        entries[f"query_{i}.jpg:ref.png"] = {
            "reference_filename": "ref.png", "success": i < n_ok, "query_2D": q2d, "reference_2D": ref2d,
            "points_3D": p3d, "num_matches": N + 2, "num_inliers": N, "inlier_mask": mask,
            "quaternion": np.array([1.0, 0.0, 0.0, 0.0]), "matrix": z["in_matrix"]}
    return z, entries


def test_reference_cache_format_roundtrip(tmp_path):
    _, entries = golden_entries()
    cache = tmp_path / "cached_matches"
    cache.mkdir()
    items = list(entries.items())
    # the reference writes one np.savez per query batch (:228-231); two files here
    np.savez(cache / "part0.npz", **dict(items[:2]))
    np.savez(cache / "part1.npz", **dict(items[2:]))
    with pytest.raises(PermissionError):
        rp.read_cached_matches(str(tmp_path))
    got = rp.read_cached_matches(str(tmp_path), trusted=True)
    assert set(got) == set(entries)
    flat = tmp_path / "matches_flat.npz"
    rp.save_flat(got, str(flat))
    back = rp.load_flat(str(flat))
    assert list(back) == list(got)
    for k, e in got.items():
        for name in rp.ENTRY_KEYS:
            a, b = e[name], back[k][name]
            if isinstance(a, np.ndarray):
                np.testing.assert_array_equal(a, b)
            else:
                assert a == b, (k, name)


def test_prediction_applies_inlier_mask():
    z, entries = golden_entries(1, 0)
    (key, e), = entries.items()
    p = rp.prediction_from_entry(e)
    N = z["in_points_3d"].shape[0]
    assert p.reference_inliers.shape == (N, 2) and p.points_3d.shape == (N, 1, 3)
    np.testing.assert_array_equal(p.reference_inliers, z["in_reference_inliers"])
    assert p.success and p.reference_filename == "ref.png" and rp.query_name(key) == "query_0.jpg"
    assert p._fields == ("success", "num_matches", "num_inliers", "reference_inliers", "query_inliers",
                         "points_3d", "quaternion", "matrix", "reference_filename", "reference_keypoints",
                         "inlier_mask")  # solve_pnp.py:7-8


def test_summary_csv_matches_reference_header(tmp_path):
    rows = [["ref.png", "q.jpg", 52, 50, 0.3, 0.29, None], ["ref.png", "q2.jpg", None, None, None, None, None]]
    rp.write_summary_csv(rows, str(tmp_path / "summary.csv"))
    with open(tmp_path / "summary.csv") as f:
        assert f.readline().strip() == REFERENCE_SUMMARY_HEADER


@pytest.mark.gpu
def test_batched_replay_reproduces_reference_feature_pnp():
    import torch
    import fmpnp
    z, entries = golden_entries(n_ok=5, n_fail=1)
    meta = json.loads(str(z["meta"]))
    q = torch.from_numpy(z["in_query"])[None]
    r = torch.from_numpy(z["in_ref"])[None]
    results, rows = rp.replay(entries, lambda name: q, {"ref.png": r}, z["in_K"], tuple(meta["image_shape"]),
                              storage=torch.float64, batch_size=2,   # three pipeline batches
                              model_kwargs=dict(n_iters=meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss,
                                                lambda_=meta["lambda0"], ratio_threshold=None))
    assert len(results) == 5 and len(rows) == 6
    for key, res in results.items():
        np.testing.assert_allclose(res["R"], z["out_R"], atol=1e-9)
        np.testing.assert_allclose(res["t"], z["out_t"], atol=1e-9)
        np.testing.assert_allclose(res["quaternion"], z["opt_quat"], atol=1e-9)
        assert res["best_num_inliers"] == int(z["best_num_inliers_"])
    failed = [row for row in rows if row[2] is None]
    assert len(failed) == 1 and failed[0][1] == "query_5.jpg"


@pytest.mark.gpu
def test_pipeline_overlap_matches_golden_and_direct_launches():
    """fmpnp.pipeline.RefinePipeline (prep stream || solve stream) over several batches gives
    the reference's feature_pnp outputs for every query of every batch."""
    import torch
    import fmpnp
    from fmpnp.pipeline import RefinePipeline
    z, entries = golden_entries(n_ok=3, n_fail=0)
    meta = json.loads(str(z["meta"]))
    q = torch.from_numpy(z["in_query"]).to("cuda:0").double()
    r = torch.from_numpy(z["in_ref"]).to("cuda:0").double()
    pred = rp.prediction_from_entry(next(iter(entries.values())))
    pipe = RefinePipeline(tuple(meta["image_shape"]), storage=torch.float64, depth=2,
                          model_kwargs=dict(n_iters=meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss,
                                            lambda_=meta["lambda0"], ratio_threshold=None))
    batches = [[(q, r, pred, z["in_K"])] * nb for nb in (2, 3, 1, 4)]
    out = pipe.run(batches)
    assert [len(b) for b in out] == [2, 3, 1, 4]
    for b in out:
        for res in b:
            np.testing.assert_allclose(res["R"], z["out_R"], atol=1e-9)
            np.testing.assert_allclose(res["t"], z["out_t"], atol=1e-9)
            assert res["best_num_inliers"] == int(z["best_num_inliers_"])


@pytest.mark.gpu
def test_gather_reference_async_matches_sync_and_flags_out_of_map():
    import torch
    from fmpnp import refine as rf
    g = torch.Generator().manual_seed(3)
    ref = torch.randn(37, 32, 32, generator=g).to("cuda:0")  # square: the reference swaps H and W scales
    inl = np.stack([np.linspace(0, 1023, 50), np.linspace(1023, 0, 50)], 1)
    a = rf.gather_reference(ref, inl, (1024, 1024), cstride=40)
    err = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    b = rf.gather_reference(ref, inl, (1024, 1024), cstride=40, err_flag=err)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and int(err.item()) == 0
    bad = inl.copy()
    bad[7] = (2000.0, 5.0)   # row/col beyond the map -> the reference raises IndexError
    with pytest.raises(IndexError):
        rf.gather_reference(ref, bad, (1024, 1024), cstride=40)
    rf.gather_reference(ref, bad, (1024, 1024), cstride=40, err_flag=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 1


@pytest.mark.gpu
def test_pipeline_raises_index_error_for_out_of_map_inliers():
    import torch
    import fmpnp
    from fmpnp.pipeline import RefinePipeline
    z, entries = golden_entries(n_ok=3, n_fail=0)
    meta = json.loads(str(z["meta"]))
    q = torch.from_numpy(z["in_query"]).to("cuda:0").double()
    pred = rp.prediction_from_entry(next(iter(entries.values())))
    r = torch.from_numpy(z["in_ref"]).to("cuda:0").double()
    bad = pred._replace(reference_inliers=np.asarray(pred.reference_inliers) + 1e6)
    pipe = RefinePipeline(tuple(meta["image_shape"]), storage=torch.float64,
                          model_kwargs=dict(n_iters=3, loss_fn=fmpnp.geman_mcclure_loss))
    with pytest.raises(IndexError):
        pipe.run([[(q, r, pred, z["in_K"])], [(q, r, bad, z["in_K"])]])


@pytest.mark.gpu
def test_pipeline_waits_for_maps_produced_on_the_callers_stream():
    """The hypercolumns are written on the caller's (current) stream by a slow chain of
    kernels immediately before run(): the pipeline's prep stream must wait for them (a
    network's output is produced exactly like this).  Every batch's poses equal the
    reference's feature_pnp outputs."""
    import torch
    import fmpnp
    from fmpnp.pipeline import RefinePipeline
    z, entries = golden_entries(n_ok=1, n_fail=0)
    meta = json.loads(str(z["meta"]))
    dev = torch.device("cuda", 0)
    q_src = torch.from_numpy(z["in_query"]).to(dev).double()
    r_src = torch.from_numpy(z["in_ref"]).to(dev).double()
    pred = rp.prediction_from_entry(next(iter(entries.values())))
    pipe = RefinePipeline(tuple(meta["image_shape"]), storage=torch.float64, depth=2,
                          model_kwargs=dict(n_iters=meta["n_iters"], loss_fn=fmpnp.geman_mcclure_loss,
                                            lambda_=meta["lambda0"], ratio_threshold=None))
    for _ in range(3):
        q = torch.full_like(q_src, float("nan"))
        r = torch.full_like(r_src, float("nan"))
        torch.cuda.synchronize()
        # ~tens of ms of work on the current stream, then the real maps land in q and r
        x = torch.randn((2048, 2048), device=dev)
        for _ in range(40):
            x = torch.tanh(x @ x * 1e-3)
        q.copy_(q_src + 0.0 * x[0, 0].double())
        r.copy_(r_src + 0.0 * x[0, 1].double())
        out = pipe.run([[(q, r, pred, z["in_K"])] * 2])
        for res in out[0]:
            np.testing.assert_allclose(res["R"], z["out_R"], atol=1e-9)
            np.testing.assert_allclose(res["t"], z["out_t"], atol=1e-9)
