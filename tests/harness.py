"""Shared test helpers: build a seeded case, run it through the HIP path
(via the drop-in `diff_gaussian_rasterization` surface) and through the
oracle, and compare."""
from __future__ import annotations

import numpy as np
import torch

from langsplatv2_amd.scenes import make_camera, make_gaussians

# Backward tolerance (documented in DESIGN.md §Parity): GPU sums per-Gaussian
# gradients in fp32 (wave reduction + atomics, arrival order varies); the
# oracle sums the identical per-pair fp32 terms sequentially in fp64.
GRAD_RTOL = 1e-5     # relative to the tensor's max |value|
GRAD_ATOL = 1e-6


def make_case(N, W, H, seed=0, sh_degree=None, lang_dim=0, quick_k=0, yaw=0.0, cov_precomp=False, device="cpu",
              bg=(0.0, 0.0, 0.0), scale_modifier=1.0):
    cam = make_camera(W, H, yaw_deg=yaw)
    g = make_gaussians(N, cam, seed=seed, sh_degree=sh_degree, lang_dim=lang_dim, quick_k=quick_k)
    if cov_precomp:
        g["cov3D_precomp"] = cov3d_torch(g["scales"] * scale_modifier, g["rotations"]).float()
        del g["scales"], g["rotations"]
    return dict(cam=cam, g=g, bg=bg, scale_modifier=scale_modifier, quick=quick_k > 0)


def cov3d_torch(s, q):
    q = q.double()
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1).view(-1, 3, 3)
    L = R @ torch.diag_embed(s.double())
    S = L @ L.transpose(1, 2)
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1)


def settings_for(case, device):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    cam, g = case["cam"], case["g"]
    quick = case["quick"]
    return GaussianRasterizationSettings(
        image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=torch.tensor(case["bg"], dtype=torch.float32, device=device), scale_modifier=case["scale_modifier"],
        viewmatrix=cam["viewmatrix"].to(device), projmatrix=cam["projmatrix"].to(device),
        sh_degree=g.get("sh_degree", 0), campos=cam["campos"].to(device), prefiltered=False, debug=False,
        include_feature=("language_feature_precomp" in g) and not quick, quick_render=quick,
        language_feature_dim=g.get("quick_dim") if quick else None)


def gpu_inputs(case, device, requires_grad=True):
    g = case["g"]
    t = {k: v.to(device) for k, v in g.items() if isinstance(v, torch.Tensor)}
    if requires_grad:
        for k in ("means3D", "shs", "colors_precomp", "opacities", "scales", "rotations", "cov3D_precomp",
                  "language_feature_precomp"):
            if k in t:
                t[k] = t[k].clone().requires_grad_(True)
    t["means2D"] = torch.zeros_like(t["means3D"], requires_grad=requires_grad)
    return t


def run_gpu_forward(case, device):
    """Forward through the library with workspace buffers decoded."""
    from langsplatv2_amd import layout, rasterizer
    rs = settings_for(case, device)
    t = gpu_inputs(case, device, requires_grad=False)
    e = torch.empty(0, device=device)
    color, lang, radii, M, bufs, _, _, _ = rasterizer._run_forward(
        t["means3D"], t.get("shs", e), t.get("colors_precomp", e), t.get("language_feature_precomp", e),
        t.get("language_feature_weights_quick", e), t.get("language_feature_indices", e), t["opacities"],
        t.get("scales", e), t.get("rotations", e), t.get("cov3D_precomp", e), rs)
    torch.cuda.synchronize()
    N = t["means3D"].shape[0]
    dec = layout.decode(bufs, N, rs.image_width, rs.image_height, M)
    out = {k: v.cpu().numpy() for k, v in dec.items()}
    out.update(color=color.cpu().numpy(), lang=lang.cpu().numpy(), radii=radii.cpu().numpy(), num_rendered=M)
    return out


def run_gpu_fwd_bwd(case, device, dout_color, dout_lang=None):
    from diff_gaussian_rasterization import GaussianRasterizer
    rs = settings_for(case, device)
    t = gpu_inputs(case, device, requires_grad=True)
    r = GaussianRasterizer(raster_settings=rs)
    kw = {}
    for k in ("shs", "colors_precomp", "scales", "rotations", "cov3D_precomp", "language_feature_precomp",
              "language_feature_weights_quick", "language_feature_indices"):
        if k in t:
            kw[k] = t[k]
    color, lang, radii = r(means3D=t["means3D"], means2D=t["means2D"], opacities=t["opacities"], **kw)
    outs, grads = [color], [torch.from_numpy(dout_color).to(device)]
    if dout_lang is not None and lang.numel() > 0 and lang.requires_grad:
        outs.append(lang)
        grads.append(torch.from_numpy(dout_lang).to(device))
    torch.autograd.backward(outs, grads)
    torch.cuda.synchronize()
    res = dict(color=color.detach().cpu().numpy(), lang=lang.detach().cpu().numpy(), radii=radii.cpu().numpy())
    for k, v in t.items():
        if isinstance(v, torch.Tensor) and v.grad is not None:
            res["grad_" + k] = v.grad.cpu().numpy()
    return res


def oracle_problem(case):
    from oracle import oracle as O
    return O.Problem(case["cam"], case["g"], bg=case["bg"], scale_modifier=case["scale_modifier"],
                     quick=case["quick"])


def assert_grad_close(name, got, ref, rtol=GRAD_RTOL, atol=GRAD_ATOL):
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    scale = max(1.0, float(np.abs(ref).max(initial=0.0)))
    err = float(np.abs(got - ref).max(initial=0.0))
    assert err <= atol + rtol * scale, f"{name}: max|err|={err:.3e} > {atol + rtol * scale:.3e} (max|ref|={scale:.3e})"
    return err, scale
