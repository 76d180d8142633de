"""The Gaussian-blur pyramid level (featurePnP/model.py:196-207 with kernel_size set).

The reference builds the kernel with kornia.filters.get_gaussian_kernel2d((k, k), (1, 1))
(kornia==0.2.2, requirements.txt:5) and blurs with a grouped conv2d, padding=1
(model.py:199-200).  kornia is not importable here, so both sides restate kornia's
published algorithm: PARITY UNPINNED against the reference.  What is pinned:
  * the façade's kernel (fmpnp.model.gaussian_kernel2d, torch fp32) against the oracle's
    (oracle.oracle.gaussian_kernel2d, numpy) and against the closed form;
  * the oracle's blur against torch's own grouped conv2d on the CPU;
  * the reference's error behaviour: even sizes raise TypeError (kornia), a level whose
    slice Python clamped (end > C) raises RuntimeError (groups = end - start channels);
  * on the GPU (-m gpu): a blurred level -- alone and after a resize -- through the façade's
    multilevel_optimization (device blur, HIP Sobel + pack, HIP LM) against the oracle's
    multilevel restatement.
"""
import math

import numpy as np
import pytest
import torch

import oracle.oracle as orc
from fmpnp.model import gaussian_blur, gaussian_kernel2d
from golden_io import case, maps64


@pytest.mark.parametrize("k", [1, 3, 5, 7])
def test_kernel_matches_oracle_and_closed_form(k):
    a = gaussian_kernel2d(k).numpy()
    b = orc.gaussian_kernel2d(k)
    assert a.dtype == np.float32 and b.dtype == np.float32
    np.testing.assert_allclose(a, b, rtol=2 ** -22, atol=0)  # fp32 exp: within an ulp
    x = np.arange(k) - k // 2
    g = np.exp(-x ** 2 / 2.0)
    np.testing.assert_allclose(a, np.outer(g, g) / g.sum() ** 2, rtol=1e-6)
    assert abs(float(a.sum(dtype=np.float64)) - 1.0) < 1e-6


def test_even_or_bad_size_raises_type_error():
    for k in (2, 4, 0, -3):
        with pytest.raises(TypeError):
            gaussian_kernel2d(k)
        with pytest.raises(TypeError):
            orc.gaussian_kernel2d(k)


@pytest.mark.parametrize("k", [3, 5])
def test_oracle_blur_equals_torch_grouped_conv(k):
    x = torch.randn((6, 13, 17), generator=torch.Generator().manual_seed(2), dtype=torch.float64)
    want = torch.nn.functional.conv2d(x[None], gaussian_kernel2d(k)[None, None].repeat(6, 1, 1, 1).double(),
                                      groups=6, padding=1)[0]
    got = orc.gaussian_blur(x.numpy(), k, 6)
    assert got.shape == (6, 13 + 3 - k, 17 + 3 - k)  # padding=1 keeps the size only for k = 3
    np.testing.assert_allclose(got, want.numpy(), rtol=0, atol=1e-15)
    np.testing.assert_allclose(gaussian_blur(x[None], k, 6)[0].numpy(), want.numpy(), rtol=0, atol=0)


def test_clamped_slice_raises_like_the_reference():
    x = torch.randn((1, 4, 9, 9), dtype=torch.float64)  # fmap[12:40] of a 16-channel map: 4 channels
    with pytest.raises(RuntimeError):
        gaussian_blur(x, 3, groups=40 - 12)
    with pytest.raises(RuntimeError):
        orc.gaussian_blur(x[0].numpy(), 3, 40 - 12)


@pytest.mark.gpu
@pytest.mark.parametrize("pyramid", [
    [(8, 16, None, 3), (0, 8, None, None)],          # blurred level, then a plain channel slice
    [(0, 8, 32, 3), (8, 16, None, None)],            # resize then blur (model.py:196-200 order)
    [(4, 12, None, 5)],                              # k = 5: padding 1 shrinks the level by 2
])
def test_blurred_level_through_facade_matches_oracle(pyramid):
    import fmpnp
    inp, meta, _ = case("pyramid3_gm")
    f, gx, gy = maps64(inp, orc.sobel)
    R, t, attrs, traces = orc.multilevel(pyramid, inp["pts3d"], inp["fref"], f, gx, gy, inp["K"],
                                         int(inp["im_width"]), int(inp["im_height"]), inp["R0"], inp["t0"], 12,
                                         0.01, "geman_mcclure", trace_cap=13)
    m = fmpnp.sparseFeaturePnP(12, loss_fn=fmpnp.geman_mcclure_loss, lambda_=0.01, storage=torch.float64)
    Rg, tg = m.multilevel_optimization(pyramid, torch.from_numpy(inp["pts3d"]), torch.from_numpy(inp["fref"]),
                                       torch.from_numpy(f), torch.from_numpy(gx), torch.from_numpy(gy),
                                       torch.from_numpy(inp["K"]), int(inp["im_width"]), int(inp["im_height"]),
                                       R_init=torch.from_numpy(inp["R0"]), t_init=torch.from_numpy(inp["t0"]),
                                       track=True)
    costs = np.concatenate([tr["cost"] for _, tr in traces])
    np.testing.assert_allclose(np.array(m.track_["costs"]), costs, rtol=1e-9)
    np.testing.assert_allclose(Rg.numpy(), R, atol=1e-8)
    np.testing.assert_allclose(tg.numpy(), t, atol=1e-8)
    assert m.best_num_inliers_ == attrs["best_num_inliers"]
    assert m.initial_cost_.item() == pytest.approx(attrs["initial_cost"], rel=1e-12)
    assert not math.isnan(m.best_cost_.item())


@pytest.mark.gpu
def test_blurred_clamped_level_raises_on_device():
    import fmpnp
    inp, meta, _ = case("pyramid3_gm")
    f, gx, gy = maps64(inp, orc.sobel)
    m = fmpnp.sparseFeaturePnP(5, loss_fn=fmpnp.geman_mcclure_loss, storage=torch.float64)
    with pytest.raises(RuntimeError):
        m.multilevel_optimization([(12, 40, None, 3)], torch.from_numpy(inp["pts3d"]), torch.from_numpy(inp["fref"]),
                                  torch.from_numpy(f), torch.from_numpy(gx), torch.from_numpy(gy),
                                  torch.from_numpy(inp["K"]), int(inp["im_width"]), int(inp["im_height"]),
                                  R_init=torch.from_numpy(inp["R0"]), t_init=torch.from_numpy(inp["t0"]))
