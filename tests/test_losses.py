"""Loss selection by the reference's names (helpers/utils.py:15-38 function names, the gin
bindings of input_configs/*.gin such as default_robotcar.gin:53 `@geman_mcclure_loss`)."""
import pytest
import torch

import fmpnp
from fmpnp import _lib, config, losses


def test_resolve_reference_functions_by_name():
    # a stand-in for helpers.utils.geman_mcclure_loss: a plain function of that name
    def geman_mcclure_loss(x):
        return x, x, x

    def squared_loss(x):
        return x, x, x
    assert losses.resolve(geman_mcclure_loss) == (_lib.GEMAN_MCCLURE, 0.0)
    assert losses.resolve(squared_loss) == (_lib.SQUARED, 0.0)
    assert losses.resolve("cauchy_loss") == (_lib.CAUCHY, 0.0)
    assert losses.resolve("huber") == (_lib.HUBER, 0.0)
    assert losses.resolve(losses.barron(1.0)) == (_lib.BARRON, 1.0)

    def unknown(x):
        return x, x, x
    with pytest.raises(ValueError):
        losses.resolve(unknown)


def test_configure_takes_gin_binding_names():
    saved = config.model_kwargs()
    try:
        config.configure(loss_fn="squared_loss")
        assert config.model_kwargs()["loss_fn"] is losses.squared_loss
        config.configure(loss_fn="geman_mcclure_loss")
        assert config.model_kwargs()["loss_fn"] is losses.geman_mcclure_loss
        config.configure(find_inliers_loss_fn="cauchy_loss")
        assert config.find_inliers_kwargs()["loss_fn"] is losses.cauchy_loss
        with pytest.raises(ValueError):
            config.configure(loss_fn="tukey_loss")
        # the facade resolves the configured loss for the device
        m = fmpnp.sparseFeaturePnP(5, loss_fn="geman_mcclure_loss")
        assert losses.resolve(m.loss_fn)[0] == _lib.GEMAN_MCCLURE
    finally:
        config.configure(loss_fn=saved["loss_fn"], find_inliers_loss_fn=losses.squared_loss)


@pytest.mark.parametrize("fn,alpha", [(losses.cauchy_loss, 0.0), (losses.geman_mcclure_loss, -2.0)])
def test_barron_forms_match_closed_forms(fn, alpha):
    x = torch.linspace(0, 10, 101, dtype=torch.float64)
    rho, d1, _ = fn(x)
    if alpha == 0.0:
        torch.testing.assert_close(rho, 2 * torch.log1p(x / 2), rtol=1e-15, atol=0)
        torch.testing.assert_close(d1, 2 / (x + 2), rtol=1e-15, atol=0)
    else:
        torch.testing.assert_close(rho, 4 * x / (x + 4), rtol=1e-14, atol=1e-15)
        torch.testing.assert_close(d1, (x / 4 + 1) ** -2, rtol=1e-14, atol=0)
