"""View-factored SH gradient of the multi-GPU exchange (dp.py).

A rank's SH coefficient gradient is basis(dir) (x) dL/dRGB, so ranks exchange
the (N, 3) clamp-masked colour gradient and their camera centre instead of the
(N, 16, 3) SH gradient, and rebuild the sum with lsr_sh_grad_from_views.

GPU: several views of one scene, each through the rasterizer backward twice —
normally (dL/dshs) and with a GradSink asking for the factored output
(dL/dRGB into `rgb_sh`) — then the rebuilt sum equals the sum of the views'
SH gradients within the harness's gradient tolerance (the render backward's
float atomics make two runs differ in the last bits), and the other
gradients of the factored run equal the normal run's within the same
tolerance.  SH degrees 1 and 3 (coefficients above the degree get 0)."""
import numpy as np
import pytest
import torch

from harness import assert_grad_close, gpu_inputs, make_case, settings_for

pytestmark = pytest.mark.gpu


def _view_grads(case, dev, yaw, factored, seed):
    from diff_gaussian_rasterization import GaussianRasterizer
    from langsplatv2_amd.rasterizer import GradSink
    from langsplatv2_amd.scenes import make_camera
    cam = make_camera(case["cam"]["W"], case["cam"]["H"], yaw_deg=yaw)
    c2 = dict(case, cam=cam)
    rs = settings_for(c2, dev)
    t = gpu_inputs(c2, dev, requires_grad=True)
    keys = ("means3D", "shs", "opacities", "scales", "rotations")
    r = GaussianRasterizer(raster_settings=rs)
    color, _, _ = r(means3D=t["means3D"], means2D=t["means2D"], opacities=t["opacities"], shs=t["shs"],
                    scales=t["scales"], rotations=t["rotations"])
    gen = torch.Generator().manual_seed(seed)
    dC = torch.randn(color.shape, generator=gen).to(dev)
    inputs = [t[k] for k in keys]
    if not factored:
        return dict(zip(keys, torch.autograd.grad([color], inputs, [dC]))), None, rs.campos
    N = t["means3D"].shape[0]
    sh_buf = torch.full(tuple(t["shs"].shape), float("nan"), device=dev)
    rgb = torch.empty((N, 3), device=dev)
    with GradSink({"shs": sh_buf}, rgb_sh=rgb):
        g = dict(zip(keys, torch.autograd.grad([color], inputs, [dC])))
    assert g["shs"].data_ptr() == sh_buf.data_ptr()          # the caller's buffer, filled by the exchange
    assert bool(torch.isnan(sh_buf).all())                  # the library left it alone
    return g, rgb, rs.campos


@pytest.mark.parametrize("deg", [1, 3])
def test_factored_sh_gradient_equals_sum_of_views(gpu, deg):
    from langsplatv2_amd import dp
    case = make_case(N=4000, W=96, H=72, seed=31, sh_degree=3)
    case["g"]["sh_degree"] = deg
    yaws = (-8.0, 0.0, 8.0)
    ref = None
    rgbs, campos = [], []
    for r, yaw in enumerate(yaws):
        full, _, _ = _view_grads(case, gpu, yaw, False, seed=r)
        fac, rgb, cp = _view_grads(case, gpu, yaw, True, seed=r)
        for k in ("means3D", "opacities", "scales", "rotations"):
            assert_grad_close(k, fac[k].cpu().numpy(), full[k].cpu().numpy())
        ref = full["shs"] if ref is None else ref + full["shs"]
        rgbs.append(rgb)
        campos.append(cp.reshape(3))
    means3D = case["g"]["means3D"].to(gpu).contiguous()
    out = torch.empty(tuple(ref.shape), device=gpu)
    dp.sh_grad_from_views(means3D, torch.stack(campos).contiguous(), torch.stack(rgbs).contiguous(), deg, out)
    got, want = out.cpu().numpy(), ref.cpu().numpy()
    nb = (deg + 1) ** 2
    assert np.all(got[:, nb:] == 0.0) and np.all(want[:, nb:] == 0.0)
    assert float(np.abs(want).max()) > 1e-3
    assert_grad_close("shs (factored)", got, want)


def test_factored_validation(gpu):
    from langsplatv2_amd import dp
    m = torch.zeros((4, 3), device=gpu)
    with pytest.raises(ValueError):
        dp.sh_grad_from_views(m, torch.zeros((2, 3), device=gpu), torch.zeros((3, 4, 3), device=gpu), 3,
                              torch.zeros((4, 16, 3), device=gpu))
    with pytest.raises(RuntimeError):   # degree 3 needs 16 coefficients
        dp.sh_grad_from_views(m, torch.zeros((1, 3), device=gpu), torch.zeros((1, 4, 3), device=gpu), 3,
                              torch.zeros((4, 4, 3), device=gpu))
