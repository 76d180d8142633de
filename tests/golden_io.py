"""Loading helpers for tests/golden/*.npz (written by tests/golden/gen_golden.py)."""
import functools
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

FORWARD_CASES = ["kat_toy6", "gm_c16", "cauchy_c16", "huber_c16", "squared_c16", "barron1_c16",
                 "ratio08_gm", "ratio05_sq", "lambda0_gm", "behind_camera_gm", "no_support_init",
                 "no_support_trial", "odd_geom_gm", "odd_geom_ratio_cauchy"]
PYRAMID_CASES = ["pyramid3_gm", "pyramid_clamp_sq", "pyramid_resize_sq", "pyramid_ratio_gm"]
ADAPTER_CASES = ["adapter_square", "adapter_nonsquare", "adapter_pyramid"]


@functools.lru_cache(maxsize=None)
def load_npz(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@functools.lru_cache(maxsize=None)
def shared_fmap(name):
    return load_npz(name)["fmap32"]


def case(name):
    """Returns (inputs dict, meta dict, golden outputs dict).

    inputs: pts3d, fref, fmap32 (float32 [C,H,W]) or fmap (fp64), optional gx/gy (fp64, the
    reference's own), K, R0, t0, im_width, im_height.
    """
    z = load_npz(name)
    meta = json.loads(str(z["meta"]))
    inp = {k[3:]: v for k, v in z.items() if k.startswith("in_")}
    if "shared_fmap" in meta:
        inp["fmap32"] = shared_fmap(meta["shared_fmap"])
    out = {k: v for k, v in z.items() if not k.startswith("in_") and k != "meta"}
    return inp, meta, out


def maps64(inp, sobel):
    """fp64 (fmap, gx, gy) for a case: stored maps if present, else fp32 map + Sobel."""
    if "fmap" in inp:
        return inp["fmap"], inp["gx"], inp["gy"]
    f = inp["fmap32"].astype(np.float64)
    gx, gy = sobel(f)
    return f, gx, gy
