"""Cached-matches replay: the reference's `--only_optimization` path.

The reference caches, per query, the sparse-to-dense matches and the PnP pose it
found (s2dhm/pose_prediction/sparse_to_dense_predictor.py:192-205 writes one
dict per "query:reference" key, :228-231 `np.savez`s them under
`<output>/cached_matches/`), and `--only_optimization` re-runs only the
feature-metric refinement from that cache (:29-39 `read_npz`, :206-223 builds a
`solve_pnp.Prediction` with the inlier mask applied), one query at a time.

Here:
  * `read_cached_matches` reads that directory.  The reference stores each entry as a
    pickled python dict inside the .npz (object arrays), so reading it executes
    pickle: the caller must pass `trusted=True` for files it produced itself;
  * `save_flat` / `load_flat` hold the same content without pickle (plain arrays and
    strings, `np.load(allow_pickle=False)`), the format this build replays from;
  * `prediction_from_entry` builds the reference's `Prediction` (same field names and
    inlier-mask application as :211-222);
  * `replay` refines many queries per device launch (the reference loops over
    queries), streamed in batches through fmpnp.pipeline, with the same per-query
    preamble as `feature_pnp`
    (optimize_feature_pnp.py:50-71: device Sobel + pack, truncating fref gather, fp64
    points, R/t from `prediction.matrix`), and returns per-query poses (t, quaternion as
    optimize_feature_pnp.py:84-91) and the reference's summary rows
    (sparse_to_dense_predictor.py:102, 257 -> `write_summary_csv`, :285).

Hypercolumns come from the caller (the CNN is outside this build): a dict or callable
mapping an image name to a [1, C, H, W] (or [C, H, W]) tensor.
"""
import os
from collections import namedtuple

import numpy as np
import torch

from . import _lib, config
from . import losses as _losses
from .matrix_utils import matrix_quaternion

# s2dhm/pose_prediction/solve_pnp.py:7-8
Prediction = namedtuple("Prediction", "success num_matches num_inliers reference_inliers query_inliers points_3d "
                                      "quaternion matrix reference_filename reference_keypoints inlier_mask")

# sparse_to_dense_predictor.py:193-204 (the cached dict's keys)
ENTRY_KEYS = ("reference_filename", "success", "query_2D", "reference_2D", "points_3D", "num_matches",
              "num_inliers", "inlier_mask", "quaternion", "matrix")
# sparse_to_dense_predictor.py:102 (result_frame columns, written with sep=";" at :285)
SUMMARY_COLUMNS = ("reference_image_origin", "query_image_origin", "num_initial_matches", "num_final_matches",
                   "initial_cost", "final_cost", "track_pickle_path")


def read_cached_matches(dirpath, trusted=False):
    """sparse_to_dense_predictor.py:29-39: every .npz under <dirpath>/cached_matches/, merged
    into {key: entry dict}.  The entries are pickled dicts: trusted=True is required."""
    if not trusted:
        raise PermissionError("the reference's cached_matches/*.npz entries are pickled python dicts; "
                              "pass trusted=True only for files you produced (or convert them with save_flat)")
    root = os.path.join(dirpath, "cached_matches")
    files = {}
    for fn in sorted(next(os.walk(root))[2]):
        with np.load(os.path.join(root, fn), allow_pickle=True) as z:
            files.update({k: z[k].item() for k in z.files})
    return files


def _flat_key(i, name):
    return f"q{i:06d}__{name}"


def save_flat(entries, path):
    """{key: entry dict} -> one pickle-free .npz (strings as unicode arrays, None omitted)."""
    arrays = {"keys": np.array(list(entries.keys()), dtype=np.str_)}
    for i, (key, e) in enumerate(entries.items()):
        for name in ENTRY_KEYS:
            v = e.get(name)
            if v is None:
                continue
            a = np.asarray(v)
            if a.dtype == object:
                raise TypeError(f"entry {key!r} field {name!r} is not a plain array")
            arrays[_flat_key(i, name)] = a
    np.savez(path, **arrays)


def load_flat(path):
    """Inverse of save_flat (np.load with allow_pickle=False)."""
    out = {}
    with np.load(path, allow_pickle=False) as z:
        keys = [str(k) for k in z["keys"]]
        for i, key in enumerate(keys):
            e = {}
            for name in ENTRY_KEYS:
                fk = _flat_key(i, name)
                if fk in z.files:
                    v = z[fk]
                    e[name] = v.item() if v.ndim == 0 else v
                else:
                    e[name] = None
            out[key] = e
    return out


def query_name(key):
    """The cache key is "query:reference" (:205); the replay reader indexes by query (:209)."""
    return key.split(":")[0]


def prediction_from_entry(e):
    """sparse_to_dense_predictor.py:210-222: the inlier mask applied to the 2D/3D points."""
    mask = np.asarray(e["inlier_mask"]).reshape(-1).astype(bool) if e.get("inlier_mask") is not None else None

    def sel(a):
        a = np.asarray(a)
        return a[mask] if mask is not None else a
    return Prediction(success=bool(e["success"]), num_matches=e["num_matches"], num_inliers=e["num_inliers"],
                      reference_inliers=sel(e["reference_2D"]), query_inliers=sel(e["query_2D"]),
                      points_3d=sel(e["points_3D"]), quaternion=e.get("quaternion"),
                      matrix=np.asarray(e["matrix"], dtype=np.float64),
                      reference_filename=e["reference_filename"], reference_keypoints=None,
                      inlier_mask=e.get("inlier_mask"))


def _hc(source, name):
    t = source(name) if callable(source) else source[name]
    t = t if isinstance(t, torch.Tensor) else torch.as_tensor(np.asarray(t))
    return t[0] if t.dim() == 4 else t


def replay(entries, query_hc, reference_hc, K, image_shape=None, storage=torch.float32, device=None,
           model_kwargs=None, sampling="nearest", batch_size=128, depth=2):
    """Refine every successful cached query, `batch_size` queries per device launch.

    entries: {key: entry dict} (read_cached_matches / load_flat).  query_hc / reference_hc:
    dict or callable, image name -> hypercolumn (loaded batch by batch, so a query set larger
    than the device holds streams through).  K: 3x3 intrinsics, or a dict / callable
    query name -> K.  Returns (results, summary rows): results[key] = dict(t, quaternion, R,
    status, initial_cost, best_cost, best_num_inliers, n_evals); summary rows in
    SUMMARY_COLUMNS order.  Unsuccessful predictions are not refined (the reference only
    refines `best_prediction.success`, :239) and get an all-None summary row (:261).
    The batches go through fmpnp.pipeline.RefinePipeline (per-query preamble of
    feature_pnp, optimize_feature_pnp.py:50-71, on one stream under the previous batch's
    LM launch on another).
    """
    from .pipeline import RefinePipeline
    cfg = config.adapter_kwargs()
    image_shape = tuple(image_shape or cfg.get("image_shape", (1024, 1024)))
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    _lib.require_device(device)
    preds = {key: prediction_from_entry(e) for key, e in entries.items()}
    keys = [key for key, pred in preds.items() if pred.success]
    bs = max(1, int(batch_size))

    def batches():
        for i in range(0, len(keys), bs):
            out = []
            for key in keys[i:i + bs]:
                pred, q = preds[key], query_name(key)
                Kq = K(q) if callable(K) else (K[q] if isinstance(K, dict) else K)
                out.append((_hc(query_hc, q), _hc(reference_hc, pred.reference_filename), pred, Kq))
            yield out

    res = []
    if keys:
        pipe = RefinePipeline(image_shape, storage=storage, device=device, depth=depth, model_kwargs=model_kwargs,
                              sampling=sampling)
        res = [r for b in pipe.run(batches()) for r in b]
    results, rows = {}, []
    by_key = dict(zip(keys, res))
    for key, pred in preds.items():
        r = by_key.get(key)
        if r is None:
            rows.append([pred.reference_filename, query_name(key), None, None, None, None, None])
            continue
        T = np.eye(4)
        T[:3, :3], T[3, :3] = r["R"], r["t"]  # optimize_feature_pnp.py:86-87 (t in the bottom row)
        results[key] = dict(t=list(r["t"]), quaternion=list(matrix_quaternion(T)), R=r["R"], status=r["status"],
                            initial_cost=r["initial_cost"], best_cost=r["best_cost"],
                            best_num_inliers=r["best_num_inliers"], n_evals=r["n_evals"])
        rows.append([pred.reference_filename, query_name(key), pred.num_matches,
                     r["best_num_inliers"] if r["has_best"] else None,
                     r["initial_cost"] if r["has_best"] else None, r["best_cost"] if r["has_best"] else None, None])
    return results, rows


def write_summary_csv(rows, path):
    """result_frame.to_csv(path, sep=";") (sparse_to_dense_predictor.py:102, 257, 285)."""
    import pandas as pd
    df = pd.DataFrame(rows, columns=list(SUMMARY_COLUMNS))
    df.to_csv(path, sep=";")
    return df


def _npy_dir_source(dirpath):
    """Image name -> hypercolumn from <dirpath>/<basename of the image>.npy (plain arrays)."""
    def load(name):
        return torch.from_numpy(np.load(os.path.join(dirpath, os.path.basename(name) + ".npy"), allow_pickle=False))
    return load


def main(argv=None):
    """python -m fmpnp.replay --matches flat.npz --hypercolumns DIR --K K.npy --out DIR
    [--image-shape 1024 1024] [--n-iters 50] [--loss geman_mcclure] [--ratio-threshold R]
    [--convert-reference-cache OUTPUT_DIR]  (trusted: reads pickled reference caches)."""
    import argparse
    ap = argparse.ArgumentParser(prog="fmpnp.replay")
    ap.add_argument("--matches", help="pickle-free matches (save_flat)")
    ap.add_argument("--convert-reference-cache", metavar="DIR",
                    help="read DIR/cached_matches/*.npz (the reference's pickled format; trusted input only) "
                         "and write --matches")
    ap.add_argument("--hypercolumns", help="directory of <image basename>.npy hypercolumns [C,H,W]")
    ap.add_argument("--K", help="3x3 intrinsics .npy")
    ap.add_argument("--image-shape", type=int, nargs=2, default=None)
    ap.add_argument("--n-iters", type=int, default=None)
    ap.add_argument("--loss", default=None)
    ap.add_argument("--ratio-threshold", type=float, default=None)
    ap.add_argument("--out", default=".")
    a = ap.parse_args(argv)
    if a.convert_reference_cache:
        save_flat(read_cached_matches(a.convert_reference_cache, trusted=True), a.matches)
        if not a.hypercolumns:
            return 0
    entries = load_flat(a.matches)
    src = _npy_dir_source(a.hypercolumns)
    kw = {}
    if a.n_iters is not None:
        kw["n_iters"] = a.n_iters
    if a.loss is not None:
        kw["loss_fn"] = _losses.by_name(a.loss)
    if a.ratio_threshold is not None:
        kw["ratio_threshold"] = a.ratio_threshold
    K = np.load(a.K, allow_pickle=False)
    results, rows = replay(entries, src, src, K, a.image_shape, model_kwargs=kw)
    os.makedirs(a.out, exist_ok=True)
    write_summary_csv(rows, os.path.join(a.out, "summary.csv"))
    with open(os.path.join(a.out, "poses.txt"), "w") as f:  # query, quaternion, t (sparse_to_dense_predictor.py:291-301)
        for key, r in results.items():
            f.write(" ".join([query_name(key)] + [repr(float(v)) for v in list(r["quaternion"]) + list(r["t"])]) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
