"""Vectorised PyTorch-CPU fp64 restatement of the reference LM loop -- TEST / BASELINE
INFRASTRUCTURE ONLY (the SURVEY.md §8d "PyTorch-CPU restatement" CPU baseline).

The same algorithm as `sparseFeaturePnP.forward` (featurePnP/model.py:245-494) with the
reference's data movement -- both evaluations per iteration, the N x C x 6 Jacobian
materialised, einsum normal equations, LU solve -- but `indexing_`'s per-point Python
loop (model.py:88-95, 82 % of the reference's run time) replaced by one
advanced-indexing gather per map.  That is what a PyTorch user would write for the
reference's CPU path, and it is what bench.py times at 1 thread and at every core of the
box beside the C restatement (oracle/fmpnp_oracle.c).

Pinned against the reference's golden vectors (tests/test_ref_torch.py).  Never imported
by the product package.
"""
import math

import torch


def _barron(x, alpha):
    """helpers/utils.py:40-78 (scale 1, first derivative)."""
    alpha = torch.as_tensor(alpha, dtype=x.dtype)
    eps = torch.tensor(torch.finfo(torch.float32).eps, dtype=x.dtype)
    beta = torch.max(eps, torch.abs(alpha - 2.0))
    asafe = torch.where(alpha >= 0, torch.ones_like(alpha), -torch.ones_like(alpha)) * torch.max(eps, alpha.abs())
    b = x / beta + 1.0
    if float(alpha) == 0.0:
        return 2 * torch.log1p(torch.min(0.5 * x, x.new_tensor(33e37))), 2 / (x + 2)
    if float(alpha) == 2.0:
        return x, torch.ones_like(x)
    return 2 * (beta / asafe) * (torch.pow(b, 0.5 * alpha) - 1.0), torch.pow(b, 0.5 * alpha - 1.0)


def loss_fn(name, alpha=0.0):
    """(rho, rho') of helpers/utils.py:15-38 by name."""
    if name == "squared":                                      # :15-17
        return lambda x: (x, torch.ones_like(x))
    if name == "huber":                                        # :19-29
        def huber(x):
            sx = torch.sqrt(x)
            isx = torch.max(sx.new_tensor(torch.finfo(torch.float32).eps), 1 / sx)
            m = x <= 1
            return torch.where(m, x, 2 * sx - 1), torch.where(m, torch.ones_like(x), isx)
        return huber
    a = {"cauchy": 0.0, "geman_mcclure": -2.0}.get(name, alpha)  # :31-38
    return lambda x: _barron(x, a)


def _project(R, t, X, K, W, H):
    """model.py:303-311: P = (R X^T)^T + t, p = round(K P / z) - 1 (int32), image mask."""
    P = torch.mm(R, X.T).T + t
    uv = torch.mm(K, P.T).T
    p2 = torch.round(uv[:, :-1] / uv[:, -1:]).to(torch.int32) - 1
    m = (p2[:, 0] >= 0) & (p2[:, 1] >= 0) & (p2[:, 0] < W) & (p2[:, 1] < H)
    return P, p2, m


def _texels(p2s, Hf, Wf, W, H):
    """indexing_'s row / column (model.py:88-89) of supported pixels p2s = (x, y)."""
    rows = (p2s[:, 1].double() * Hf / H).floor().long()
    cols = (p2s[:, 0].double() * Wf / W).floor().long()
    return rows, cols


def _skew(v):
    z = torch.zeros_like(v[:, 0])
    return torch.stack([z, -v[:, 2], v[:, 1], v[:, 2], z, -v[:, 0], -v[:, 1], v[:, 0], z], -1).reshape(-1, 3, 3)


def _so3exp(w):
    """helpers/utils.py:209-221."""
    theta = w.norm()
    Wm = _skew((w / theta)[None])[0]
    res = Wm * torch.sin(theta) + (Wm @ Wm) * (1 - torch.cos(theta))
    if theta < 1e-12:
        res = torch.zeros_like(res)
    return torch.eye(3, dtype=w.dtype) + res


def forward(pts3d, fref, fmap, gx, gy, K, W, H, R0, t0, n_iters=50, lambda_=0.01, loss="squared",
            ratio_threshold=None, barron_alpha=0.0):
    """sparseFeaturePnP.forward (model.py:245-494) on fp64 CPU tensors.  Returns
    (R_best, t_best, info) with info = best_cost, best_num_inliers, costs (tracked)."""
    X, fref, fmap, gx, gy, K = (torch.as_tensor(a, dtype=torch.float64) for a in (pts3d, fref, fmap, gx, gy, K))
    R, t = torch.as_tensor(R0, dtype=torch.float64), torch.as_tensor(t0, dtype=torch.float64)
    Hf, Wf = fmap.shape[-2:]
    rho_fn = loss_fn(loss, barron_alpha)
    fx, fy = K[0, 0], K[1, 1]
    lam, lr = lambda_, 1.0
    R_best, t_best = R, t
    info = dict(best_cost=None, best_num_inliers=None, costs=[])

    def residual(R, t):
        P, p2, m = _project(R, t, X, K, W, H)
        if not bool(m.any()):
            return None
        rows, cols = _texels(p2[m], Hf, Wf, W, H)
        e = fmap[:, rows, cols].T - fref[m]                        # model.py:322 (indexing_ in one gather)
        keep = None
        if ratio_threshold is not None:                            # model.py:324-336
            c_full, _ = rho_fn(0.5 * (e ** 2).sum(-1))
            keep = torch.abs(c_full) < torch.max(torch.abs(c_full)) * ratio_threshold
            e, P_s, rows, cols = e[keep], P[m][keep], rows[keep], cols[keep]
        else:
            P_s = P[m]
        rho, w = rho_fn(0.5 * (e ** 2).sum(-1))                    # model.py:338-339
        return rho, w, e, P_s, rows, cols

    prev = None
    for i in range(n_iters):
        r = residual(R, t)
        if r is None:                                              # model.py:316-320
            return R, t, info
        rho, w, e, P, rows, cols = r
        if i == 0:                                                 # model.py:347-359
            prev = rho.mean(-1)
            info.update(best_cost=prev, best_num_inliers=P.shape[0])
            info["costs"].append(float(prev))
        # Jacobian chain, materialised as the reference does (model.py:369-394)
        n = P.shape[0]
        J_p_T = torch.cat([torch.eye(3, dtype=torch.float64)[None].repeat(n, 1, 1), -_skew(P)], -1)
        o, z = torch.ones(n, dtype=torch.float64), torch.zeros(n, dtype=torch.float64)
        J_px_p = torch.stack([fx * o, z, -fx * P[:, 0] / P[:, 2], z, fy * o, -fy * P[:, 1] / P[:, 2]],
                             -1).reshape(n, 2, 3) / P[:, 2, None, None]
        J_f_px = torch.stack([gx[:, rows, cols].T, gy[:, rows, cols].T], -1)
        J = J_f_px @ J_px_p @ J_p_T
        g = (w[:, None] * torch.einsum("bij,bi->bj", J, e)).sum(-2)          # model.py:397-399
        Hs = (w[:, None, None] * torch.einsum("ijk,ijl->ikl", J, J)).sum(-3)  # model.py:403-405
        if lam:                                                     # optimizer_step, model.py:46-48
            Hs = Hs + (Hs.diagonal() + 1e-9).diag_embed() * lam
        LU, piv = torch.linalg.lu_factor(Hs)                        # model.py:51,61
        delta = -lr * torch.linalg.lu_solve(LU, piv, g[:, None])[:, 0]
        if torch.isnan(delta).any():                                # model.py:411-413
            break
        dR = _so3exp(delta[3:])                                     # model.py:416-426
        R_new, t_new = dR @ R, dR @ t + delta[:3]
        r2 = residual(R_new, t_new)                                 # model.py:428-462
        if r2 is None:
            return R, t, info
        new_cost = r2[0].mean()
        info["costs"].append(float(new_cost))
        worse = bool(new_cost > prev)
        lam = min(max(lam * (10 if worse else 1 / 10), 1e-6), 1e4)  # model.py:469-470
        if worse:                                                    # model.py:472-476
            lr = min(max(0.1 * lr, 1e-3), 1.0)
            continue
        lr = 1.0
        if new_cost < info["best_cost"]:                            # model.py:477-483
            R_best, t_best = R_new, t_new
            info.update(best_cost=new_cost, best_num_inliers=r2[3].shape[0])
        prev = new_cost
        R, t = R_new, t_new
    return R_best, t_best, info


def sobel(x):
    """Vendored kornia Sobel (featurePnP/helpers/sobel_pytorch.py): unnormalised, zero padded."""
    x = torch.as_tensor(x, dtype=torch.float64)
    kx = torch.tensor([[-1.0, 0.0, 1.0], [-2.0, 0.0, 2.0], [-1.0, 0.0, 1.0]], dtype=torch.float64)
    k = torch.stack([kx, kx.T])[:, None]                            # [2,1,3,3]
    g = torch.nn.functional.conv2d(x[:, None], k, padding=1)        # [C,2,H,W]
    return g[:, 0].contiguous(), g[:, 1].contiguous()


def rot_angle(Ra, Rb):
    c = (float(torch.trace(torch.as_tensor(Ra).T @ torch.as_tensor(Rb))) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))
