"""CPU checks of the RGB-phase loop helpers (langsplatv2_amd/train_loop.py):
the SH ramp at window granularity (train.py:135-136), the per-view
bookkeeping (train.py:250-251, scene/gaussian_model.py:506-508) and the SSIM /
L1 loss restatement (utils/loss_utils.py:18-75).  The GPU path (two ranks
through the HIP rasterizer) is tests/test_0_train_dp.py."""
import math

import torch

from langsplatv2_amd import dp
from langsplatv2_amd.train_loop import GaussianState, apply_view_stats, l1_loss, sh_ramp, ssim, view_loss


def _state(n=5):
    g = torch.Generator().manual_seed(0)
    return GaussianState(torch.randn(n, 3, generator=g), torch.randn(n, 16, 3, generator=g),
                         torch.rand(n, 1, generator=g) * 0.9 + 0.05, torch.rand(n, 3, generator=g) + 0.1,
                         torch.randn(n, 4, generator=g))


def test_activations_round_trip():
    g = torch.Generator().manual_seed(1)
    op = torch.rand(7, 1, generator=g) * 0.9 + 0.05
    sc = torch.rand(7, 3, generator=g) + 0.1
    gs = GaussianState(torch.zeros(7, 3), torch.zeros(7, 16, 3), op, sc, torch.randn(7, 4, generator=g))
    torch.testing.assert_close(gs.get_opacity, op, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(gs.get_scaling, sc, rtol=1e-6, atol=0)
    assert gs.get_features.shape == (7, 16, 3)
    torch.testing.assert_close(gs.get_rotation.norm(dim=1), torch.ones(7))


def test_sh_ramp_windows():
    gs = _state()
    # one rank, the reference's per-iteration rule: degree d after iteration 1000 d
    for it in range(0, 4000):
        sh_ramp(gs, it, 1, 1000)
        assert gs.active_sh_degree == min(3, (it + 1) // 1000)
    gs = _state()
    sh_ramp(gs, 0, 8, 4)        # window 1..8 crosses 4 and 8: two steps up
    assert gs.active_sh_degree == 2
    sh_ramp(gs, 8, 8, 4)        # capped at the maximum degree
    assert gs.active_sh_degree == 3


def test_view_stats_match_per_view_updates():
    gs = _state()
    grads = [torch.tensor([[3.0, 4.0, 9.0]] * 5), torch.tensor([[0.0, 1.0, 0.0]] * 5)]
    radii = [torch.tensor([2, 0, 5, 1, 0], dtype=torch.int32), torch.tensor([4, 3, 0, 0, 0], dtype=torch.int32)]
    for gr, r in zip(grads, radii):
        apply_view_stats(gs, r, dp.densify_increment(gr, r))
    assert gs.max_radii2D.tolist() == [4.0, 3.0, 5.0, 1.0, 0.0]
    assert gs.denom.squeeze(1).tolist() == [2.0, 1.0, 1.0, 1.0, 0.0]
    assert gs.xyz_gradient_accum.squeeze(1).tolist() == [6.0, 1.0, 5.0, 5.0, 0.0]


def test_ssim_and_l1():
    g = torch.Generator().manual_seed(2)
    a = torch.rand(3, 24, 32, generator=g)
    assert abs(float(ssim(a, a)) - 1.0) < 1e-6
    b = (a + 0.1 * torch.randn(3, 24, 32, generator=g)).clamp(0, 1)
    s = float(ssim(a, b))
    assert 0.0 < s < 1.0
    assert math.isclose(float(l1_loss(a, b)), float((a - b).abs().mean()), rel_tol=1e-7)
    assert math.isclose(float(view_loss(a, b, 0.2)), 0.8 * float(l1_loss(a, b)) + 0.2 * (1 - s), rel_tol=1e-6)


def test_ssim_l1_match_reference_golden():
    """Vectors from the reference's own utils/loss_utils.py (tests/golden/make_ref_ssim.py)."""
    import os
    import numpy as np
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_ssim.npz"))
    for i in range(3):
        a, b = torch.from_numpy(z[f"a{i}"]), torch.from_numpy(z[f"b{i}"])
        assert abs(float(ssim(a, b)) - float(z[f"ssim{i}"])) < 1e-6
        assert abs(float(l1_loss(a, b)) - float(z[f"l1_{i}"])) < 1e-7
