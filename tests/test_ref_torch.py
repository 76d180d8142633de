"""The PyTorch-CPU restatement (oracle/ref_torch.py, bench.py's second CPU baseline) against
the reference's own golden vectors: same trajectory (tracked costs), same result.  CPU only."""
import numpy as np
import pytest
import torch

from golden_io import FORWARD_CASES, case, maps64
from oracle import ref_torch

# every forward case except the early exits' attribute bookkeeping (checked in the C oracle)
CASES = [c for c in FORWARD_CASES]


@pytest.mark.parametrize("name", CASES)
def test_ref_torch_matches_reference(name):
    inp, meta, gold = case(name)
    f, gx, gy = maps64(inp, lambda x: tuple(a.numpy() for a in ref_torch.sobel(x)))
    R, t, info = ref_torch.forward(inp["pts3d"], inp["fref"], f, gx, gy, inp["K"], int(inp["im_width"]),
                                   int(inp["im_height"]), inp["R0"], inp["t0"], meta["n_iters"], meta["lambda0"],
                                   meta["loss"], meta.get("ratio_threshold"), meta.get("barron_alpha") or 0.0)
    np.testing.assert_allclose(R.numpy(), gold["out_R"], atol=1e-9)
    np.testing.assert_allclose(t.numpy(), gold["out_t"], atol=1e-9)
    if "track_costs" in gold:
        np.testing.assert_allclose(info["costs"], gold["track_costs"], rtol=1e-10)
    if bool(gold["has_best_cost_"]):
        assert float(info["best_cost"]) == pytest.approx(float(gold["best_cost_"]), rel=1e-10)
        assert info["best_num_inliers"] == int(gold["best_num_inliers_"])


def test_ref_torch_sobel_matches_oracle():
    import oracle.oracle as orc
    x = torch.randn((5, 17, 23), generator=torch.Generator().manual_seed(1), dtype=torch.float64).numpy()
    gx, gy = ref_torch.sobel(x)
    ogx, ogy = orc.sobel(x)
    np.testing.assert_allclose(gx.numpy(), ogx, atol=1e-13)
    np.testing.assert_allclose(gy.numpy(), ogy, atol=1e-13)
