"""Synthetic refinement problems (SURVEY.md §8d recipe) for benches and tests.

There is no dataset or CNN checkpoint offline, so the hypercolumn is a smoothed,
L2-normalised random field of the reference's shape and dtype (fp32,
L2-normalised over channels like network.py:172-173).  Image size = 4x the
feature map (stride 4), K = [[0.8 W, 0, W/2], [0, 0.8 W, H/2], [0, 0, 1]],
points uniformly inside the central 80 % of the image at depth U(5, 25),
reference descriptors = the nearest-texel gather at the identity pose, initial
pose Rz(1 deg), t = (0.05, -0.03, 0.10).
"""
import math
from collections import namedtuple

import numpy as np
import torch

from .refine import project_pixels


def rot_z(deg):
    a = math.radians(deg)
    return np.array([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]])


def feature_map(C, Hf, Wf, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    x = torch.randn((1, C, Hf, Wf), generator=g, device=device, dtype=torch.float32)
    x = torch.nn.functional.avg_pool2d(x, 7, stride=1, padding=3)
    x = x / x.norm(dim=1, keepdim=True).clamp_min(1e-12)
    return x[0].contiguous()


def scene(N, Hf, Wf, seed):
    rng = np.random.Generator(np.random.PCG64(int(seed) + 1000003))
    W, H = 4 * Wf, 4 * Hf
    K = np.array([[0.8 * W, 0.0, W / 2.0], [0.0, 0.8 * W, H / 2.0], [0.0, 0.0, 1.0]])
    u = rng.uniform(0.1, 0.9, N) * W
    v = rng.uniform(0.1, 0.9, N) * H
    z = rng.uniform(5.0, 25.0, N)
    X = np.stack([(u - K[0, 2]) * z / K[0, 0], (v - K[1, 2]) * z / K[1, 1], z], 1)
    return X, K, W, H


def reference_descriptors(fmap, X, K, W, H):
    """fref = NN gather at the identity pose (model.py:74-97 conventions), [N, C] like fmap."""
    p = project_pixels(np.eye(3), np.zeros(3), X, K)
    inside = (p[:, 0] >= 0) & (p[:, 1] >= 0) & (p[:, 0] < W) & (p[:, 1] < H)
    assert inside.all()
    C, Hf, Wf = fmap.shape
    rows = torch.as_tensor((p[:, 1].astype(np.int64) * Hf) // H, device=fmap.device)
    cols = torch.as_tensor((p[:, 0].astype(np.int64) * Wf) // W, device=fmap.device)
    return fmap[:, rows, cols].T.contiguous()


def rot_xyz(dx, dy, dz):
    """Rz(dz) Ry(dy) Rx(dx), degrees (the golden vectors' harder initial rotations)."""
    ax, ay = math.radians(dx), math.radians(dy)
    rx = np.array([[1.0, 0.0, 0.0], [0.0, math.cos(ax), -math.sin(ax)], [0.0, math.sin(ax), math.cos(ax)]])
    ry = np.array([[math.cos(ay), 0.0, math.sin(ay)], [0.0, 1.0, 0.0], [-math.sin(ay), 0.0, math.cos(ay)]])
    return rot_z(dz) @ ry @ rx


# initial poses: "easy" = SURVEY.md §8d (Rz(1 deg), t = (0.05, -0.03, 0.10)); "hard" = the
# golden vectors' perturbation (tests/golden/gen_golden.py: rot_xyz(0.6, -0.4, 2.0),
# t = (0.2, -0.12, 0.35)), several texels of image motion per point
INITS = {"easy": (rot_z(1.0), np.array([0.05, -0.03, 0.10])),
         "hard": (rot_xyz(0.6, -0.4, 2.0), np.array([0.2, -0.12, 0.35]))}


def problem_inputs(N=512, C=256, Hf=240, Wf=320, seed=0, device="cuda", init="easy"):
    """Dict of one query's inputs: fmap [C,Hf,Wf] fp32 (device), fref [N,C] fp32 (device),
    pts3d [N,3] fp64 (numpy), K, im_width, im_height, R0, t0."""
    fmap = feature_map(C, Hf, Wf, seed, device)
    X, K, W, H = scene(N, Hf, Wf, seed)
    fref = reference_descriptors(fmap, X, K, W, H)
    R0, t0 = INITS[init]
    return dict(fmap=fmap, fref=fref, pts3d=X, K=K, im_width=W, im_height=H, R0=R0.copy(), t0=t0.copy())


# the reference's Prediction fields feature_pnp reads (s2dhm/pose_prediction/solve_pnp.py:7-8)
QueryPrediction = namedtuple("QueryPrediction", "points_3d reference_inliers matrix")


def pipeline_queries(n_batches, batch, N=512, C=256, Hf=240, Wf=320, device="cuda", seed0=0, init="easy"):
    """Batches of feature_pnp-style queries (query_hc, reference_hc, prediction, K) for
    fmpnp.pipeline.RefinePipeline, and the image_shape (W, H) they use.  The reference
    hypercolumn is the query map; the reference inliers are placed so that the reference's
    gather (optimize_feature_pnp.py:51-56: row = trunc(y * W_ref / image_shape[1]),
    col = trunc(x * H_ref / image_shape[0])) picks each point's identity-pose texel, i.e.
    the same descriptors as reference_descriptors()."""
    batches = []
    W, H = 4 * Wf, 4 * Hf
    for b in range(n_batches):
        qs = []
        for i in range(batch):
            seed = seed0 + 1000 * b + i
            fmap = feature_map(C, Hf, Wf, seed, device)
            X, K, _, _ = scene(N, Hf, Wf, seed)
            p = project_pixels(np.eye(3), np.zeros(3), X, K)
            rows = (p[:, 1].astype(np.int64) * Hf) // H
            cols = (p[:, 0].astype(np.int64) * Wf) // W
            inl = np.stack([(cols + 0.5) * W / Hf, (rows + 0.5) * H / Wf], 1)
            T = np.eye(4)
            T[:3, :3], T[:3, 3] = INITS[init]
            qs.append((fmap, fmap[None], QueryPrediction(X, inl, T), K))
        batches.append(qs)
    return batches, (W, H)
