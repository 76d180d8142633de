"""Robust losses with the reference's call signature (featurePnP/helpers/utils.py:15-78).

Each function maps x = 0.5 * ||e||^2 to (rho, rho', rho'') like the reference, so
code that calls them directly keeps working.  The refiner itself never calls
them: `sparseFeaturePnP` reads the `fmpnp_loss` tag and the HIP kernel evaluates
the same formulas in fp64 on the device (csrc/fmpnp_device.h:loss_eval).
"""
import torch

from . import _lib

_EPS32 = torch.finfo(torch.float32).eps


def _tag(fn, code, alpha=0.0):
    fn.fmpnp_loss = code
    fn.fmpnp_alpha = float(alpha)
    return fn


def squared_loss(x):
    """utils.py:15-17."""
    return x, torch.ones_like(x), torch.zeros_like(x)


def huber_loss(x):
    """utils.py:19-29 (threshold 1)."""
    mask = x <= 1
    sx = torch.sqrt(x)
    isx = torch.maximum(sx.new_tensor(_EPS32), 1 / sx)
    loss = torch.where(mask, x, 2 * sx - 1)
    d1 = torch.where(mask, torch.ones_like(x), isx)
    d2 = torch.where(mask, torch.zeros_like(x), -isx / (2 * x))
    return loss, d1, d2


def barron_loss(x, alpha):
    """utils.py:40-78: general robust loss on an already squared input (scale 1)."""
    alpha = torch.as_tensor(alpha, dtype=x.dtype, device=x.device)
    eps = torch.tensor(_EPS32, dtype=x.dtype, device=x.device)
    beta = torch.maximum(eps, torch.abs(alpha - 2.0))
    asafe = torch.where(alpha >= 0, torch.ones_like(alpha), -torch.ones_like(alpha)) * torch.maximum(eps, alpha.abs())
    l_two, d_two = x, torch.ones_like(x)
    l_zero = 2 * torch.log1p(torch.minimum(0.5 * x, x.new_tensor(33e37)))
    d_zero = 2 / (x + 2)
    b = x / beta + 1.0
    l_other = 2 * (beta / asafe) * (torch.pow(b, 0.5 * alpha) - 1.0)
    d_other = torch.pow(b, 0.5 * alpha - 1.0)
    loss = torch.where(alpha == 0, l_zero, torch.where(alpha == 2, l_two, l_other))
    d1 = torch.where(alpha == 0, d_zero, torch.where(alpha == 2, d_two, d_other))
    return loss, d1, torch.zeros_like(x)


def cauchy_loss(x):
    """utils.py:31-34 (Barron alpha = 0)."""
    return barron_loss(x, 0.0)


def geman_mcclure_loss(x):
    """utils.py:36-38 (Barron alpha = -2)."""
    return barron_loss(x, -2.0)


def barron(alpha):
    """A Barron loss with a fixed alpha, usable as sparseFeaturePnP(loss_fn=...)."""
    a = float(alpha)
    return _tag(lambda x: barron_loss(x, a), _lib.BARRON, a)


def scaled_loss(x, fn, a):
    """utils.py:10-13 (unused by the LM loop; kept for API completeness)."""
    a2 = a ** 2
    loss, d1, d2 = fn(x / a2)
    return loss * a2, d1, d2 / a2


_tag(squared_loss, _lib.SQUARED)
_tag(huber_loss, _lib.HUBER)
_tag(cauchy_loss, _lib.CAUCHY)
_tag(geman_mcclure_loss, _lib.GEMAN_MCCLURE)

BY_NAME = {"squared": squared_loss, "huber": huber_loss, "cauchy": cauchy_loss,
           "geman_mcclure": geman_mcclure_loss}


def by_name(name):
    """The loss for a short name ("geman_mcclure") or the reference's function / gin binding
    name ("geman_mcclure_loss", helpers/utils.py:15-38, default_robotcar.gin:53)."""
    key = name[:-len("_loss")] if name.endswith("_loss") else name
    if key not in BY_NAME:
        raise ValueError(f"unknown loss {name!r}: one of {sorted(BY_NAME)} (optionally with the '_loss' suffix)")
    return BY_NAME[key]


def resolve(loss_fn):
    """(loss code, alpha) of a loss function; only the losses above run on the device."""
    if isinstance(loss_fn, str):
        loss_fn = by_name(loss_fn)
    code = getattr(loss_fn, "fmpnp_loss", None)
    if code is None:
        # the reference's own helpers.utils functions: squared_loss, huber_loss, cauchy_loss,
        # geman_mcclure_loss (utils.py:15-38)
        name = getattr(loss_fn, "__name__", "")
        try:
            return by_name(name).fmpnp_loss, 0.0
        except ValueError:
            raise ValueError(f"unsupported loss_fn {loss_fn!r}: use fmpnp.losses.{{squared,huber,cauchy,"
                             f"geman_mcclure}}_loss or fmpnp.losses.barron(alpha)") from None
    return code, getattr(loss_fn, "fmpnp_alpha", 0.0)
