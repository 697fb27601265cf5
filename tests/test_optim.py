"""Fused Adam (csrc/adam.hip, langsplatv2_amd.optim).

CPU: the float64 oracle restatement against torch.optim.Adam itself (the
reference's optimizer class, scene/gaussian_model.py:255).  GPU: FusedAdam
against torch.optim.Adam on the same device and against the oracle, over
several steps, several parameter groups (the reference's named groups and
lr = 0.0 default), weight decay, and a length that exercises the scalar tail.
Tolerance: 2e-6 relative to max |param| (fp32 elementwise rounding order
differs from torch's multi-pass foreach kernels).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

RTOL = 2e-6


def _close(got, ref, what):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-12)
    assert err <= RTOL, f"{what}: relative error {err:.3g}"


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_oracle_matches_torch_adam(wd):
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(1000, generator=g, dtype=torch.float64)
    grads = [torch.randn(1000, generator=g, dtype=torch.float64) for _ in range(4)]
    p = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p], lr=0.01, eps=1e-15, weight_decay=wd)
    for gr in grads:
        p.grad = gr.clone()
        opt.step()
    ref_p, ref_m, ref_v = O.adam_steps(p0.numpy(), [x.numpy() for x in grads], 0.01, eps=1e-15, weight_decay=wd)
    np.testing.assert_allclose(p.detach().numpy(), ref_p, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(opt.state[p]["exp_avg"].numpy(), ref_m, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(opt.state[p]["exp_avg_sq"].numpy(), ref_v, rtol=1e-12, atol=1e-15)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,wd", [((100_003,), 0.0), ((4096, 64), 0.0), ((1, 64, 512), 0.02)])
def test_fused_adam_matches_torch(shape, wd):
    from langsplatv2_amd.optim import FusedAdam
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(1)
    init = [torch.randn(shape, generator=g), torch.randn(shape, generator=g)]
    grads = [[torch.randn(shape, generator=g) for _ in range(5)] for _ in init]
    ps_t = [x.to(dev).requires_grad_(True) for x in init]
    ps_f = [x.to(dev).requires_grad_(True) for x in init]
    groups = lambda ps: [{"params": [ps[0]], "lr": 0.0025, "name": "language_feature"},   # noqa: E731
                         {"params": [ps[1]], "lr": 0.016, "name": "xyz"}]
    ot = torch.optim.Adam(groups(ps_t), lr=0.0, eps=1e-15, weight_decay=wd)
    of = FusedAdam(groups(ps_f), lr=0.0, eps=1e-15, weight_decay=wd)
    for s in range(5):
        for i in range(2):
            ps_t[i].grad = grads[i][s].to(dev)
            ps_f[i].grad = grads[i][s].to(dev)
        ot.step()
        of.step()
    for i, lr in enumerate((0.0025, 0.016)):
        _close(ps_f[i].detach().cpu(), ps_t[i].detach().cpu(), f"param {i} vs torch")
        _close(of.state[ps_f[i]]["exp_avg"].cpu(), ot.state[ps_t[i]]["exp_avg"].cpu(), f"exp_avg {i}")
        _close(of.state[ps_f[i]]["exp_avg_sq"].cpu(), ot.state[ps_t[i]]["exp_avg_sq"].cpu(), f"exp_avg_sq {i}")
        ref_p, _, _ = O.adam_steps(init[i].numpy(), [x.numpy() for x in grads[i]], lr, eps=1e-15, weight_decay=wd)
        _close(ps_f[i].detach().cpu(), ref_p, f"param {i} vs oracle")
    assert float(of.state[ps_f[0]]["step"]) == 5.0


@pytest.mark.gpu
def test_fused_adam_state_surgery_like_densification():
    """The reference replaces / prunes a parameter and its exp_avg / exp_avg_sq
    in the optimizer state (scene/gaussian_model.py:352-420); FusedAdam keeps
    working on the new tensors."""
    from langsplatv2_amd.optim import FusedAdam
    dev = torch.device("cuda:0")
    p = torch.nn.Parameter(torch.randn(1000, 3, device=dev))
    opt = FusedAdam([{"params": [p], "lr": 0.01, "name": "xyz"}], lr=0.0, eps=1e-15)
    p.grad = torch.randn_like(p)
    opt.step()
    keep = torch.arange(1000, device=dev) % 3 != 0
    st = opt.state.pop(p)
    st["exp_avg"] = st["exp_avg"][keep].contiguous()
    st["exp_avg_sq"] = st["exp_avg_sq"][keep].contiguous()
    q = torch.nn.Parameter(p.detach()[keep].contiguous())
    opt.param_groups[0]["params"][0] = q
    opt.state[q] = st
    q.grad = torch.randn_like(q)
    before = q.detach().clone()
    opt.step()
    assert torch.isfinite(q).all() and not torch.equal(before, q.detach())
    assert float(opt.state[q]["step"]) == 2.0
