"""The drop-in boundary exercised with the reference's exact call pattern.

`render()` (/root/reference/gaussian_renderer/__init__.py:19-129) is the only
caller of the rasterizer.  What it does that a plain call does not:
  * means2D = torch.zeros_like(xyz, requires_grad=True) + 0 — a NON-LEAF
    tensor — plus retain_grad(), and later reads means2D.grad[:, :2]
    (scene/gaussian_model.py:506-508) (:27-31);
  * settings built by keyword with debug / include_feature / quick_render from
    the pipe / opt objects (:37-52);
  * cov3D from Python when pipe.compute_cov3D_python (:62-69), colours from
    eval_sh + 0.5, clamp_min(0) when pipe.convert_SHs_python (:74-81);
  * torch.zeros((1,)) placeholders for the unused language inputs in all
    three modes (:87-103) — quick mode with include_feature ALSO set
    (eval_lerf.sh:23-25);
  * returns radii > 0 as the visibility filter, used with
    torch.max(max_radii2D[vis], radii[vis]) (:125-129, train.py:250).
`render_like_reference` below restates that sequence (test code; the
reference is not importable on the GPU box) and every mode is compared with
the oracle: forward bit-exact, gradients within tests/harness.py's tolerance.
"""
import math
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from harness import FWD_ATOL_FX, assert_grad_close, assert_img, cov3d_torch, make_case
from test_oracle import sh_eval_t

pytestmark = pytest.mark.gpu


class _Model:
    """The attributes render() reads from GaussianModel (scene/gaussian_model.py)."""

    def __init__(self, g, dev, sh_degree, logits=None, quick=None):
        self.xyz = g["means3D"].to(dev).clone().requires_grad_(True)
        self.opacity = g["opacities"].to(dev).clone().requires_grad_(True)
        self.scaling = g["scales"].to(dev).clone().requires_grad_(True)
        self.rotation = g["rotations"].to(dev).clone().requires_grad_(True)
        self.features = g["shs"].to(dev).clone().requires_grad_(True)
        self.active_sh_degree = sh_degree
        self.max_sh_degree = 3
        self.logits = None if logits is None else logits.to(dev).clone().requires_grad_(True)
        self._language_feature_weights = None if quick is None else quick[0].to(dev)
        self._language_feature_indices = None if quick is None else quick[1].to(dev)

    get_xyz = property(lambda self: self.xyz)
    get_opacity = property(lambda self: self.opacity)
    get_scaling = property(lambda self: self.scaling)
    get_rotation = property(lambda self: self.rotation)
    get_features = property(lambda self: self.features)

    def get_covariance(self, scaling_modifier=1.0):
        return cov3d_torch(self.scaling * scaling_modifier, self.rotation).float()

    def get_render_weights(self, topk):
        from langsplatv2_amd import lang_codes
        return lang_codes.get_render_weights(self.logits, 1, 64, topk)


def _camera(W, H, yaw=0.0):
    from langsplatv2_amd.scenes import make_camera
    c = make_camera(W, H, yaw_deg=yaw)
    return SimpleNamespace(FoVx=2 * math.atan(c["tanfovx"]), FoVy=2 * math.atan(c["tanfovy"]), image_width=W,
                           image_height=H, world_view_transform=c["viewmatrix"], full_proj_transform=c["projmatrix"],
                           camera_center=c["campos"], _cam=c)


def render_like_reference(cam, pc, pipe, bg_color, opt, scaling_modifier=1.0, override_color=None):
    """The call sequence of gaussian_renderer/__init__.py:19-129 (restated)."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    dev = pc.get_xyz.device
    screenspace_points = torch.zeros_like(pc.get_xyz, dtype=pc.get_xyz.dtype, requires_grad=True, device=dev) + 0
    screenspace_points.retain_grad()
    settings = GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), bg=bg_color,
        scale_modifier=scaling_modifier, viewmatrix=cam.world_view_transform.to(dev),
        projmatrix=cam.full_proj_transform.to(dev), sh_degree=pc.active_sh_degree,
        campos=cam.camera_center.to(dev), prefiltered=False, debug=pipe.debug,
        include_feature=opt.include_feature, quick_render=opt.quick_render)
    rasterizer = GaussianRasterizer(raster_settings=settings)
    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales, rotations = pc.get_scaling, pc.get_rotation
    shs = colors_precomp = None
    if override_color is None:
        if pipe.convert_SHs_python:
            dirs = pc.get_xyz - cam.camera_center.to(dev).repeat(pc.get_features.shape[0], 1)
            dirs = dirs / dirs.norm(dim=1, keepdim=True)
            colors_precomp = torch.clamp_min(sh_eval_t(pc.active_sh_degree, pc.get_features, dirs) + 0.5, 0.0)
        else:
            shs = pc.get_features
    else:
        colors_precomp = override_color
    z1 = lambda: torch.zeros((1,), dtype=pc.get_opacity.dtype, device=dev)  # noqa: E731
    if opt.quick_render:
        lw, lwq, li = z1(), pc._language_feature_weights, pc._language_feature_indices
    elif opt.include_feature:
        lw, lwq, li = pc.get_render_weights(opt.topk), z1(), z1()
    else:
        lw, lwq, li = z1(), z1(), z1()
    image, lmap, radii = rasterizer(means3D=pc.get_xyz, means2D=screenspace_points, shs=shs,
                                    colors_precomp=colors_precomp, language_feature_precomp=lw,
                                    language_feature_weights_quick=lwq, language_feature_indices=li,
                                    opacities=pc.get_opacity, scales=scales, rotations=rotations,
                                    cov3D_precomp=cov3D_precomp)
    return {"render": image, "language_feature_weight_map": lmap, "viewspace_points": screenspace_points,
            "visibility_filter": radii > 0, "radii": radii, "_lw": lw, "_colors": colors_precomp,
            "_cov": cov3D_precomp}


def _setup(mode, dev, N=3000, W=112, H=96, seed=11):
    case = make_case(N=N, W=W, H=H, sh_degree=3, seed=seed, quick_k=4 if mode == "quick" else 0)
    g = case["g"]
    logits = torch.randn(N, 64, generator=torch.Generator().manual_seed(seed)) if mode == "feature" else None
    quick = (g["language_feature_weights_quick"], g["language_feature_indices"]) if mode == "quick" else None
    pc = _Model(g, dev, 3, logits=logits, quick=quick)
    return case, pc, _camera(W, H)


def _oracle(case, pc, extra, quick=False, bg=(0.0, 0.0, 0.0)):
    from oracle import oracle as O
    g = dict(case["g"])
    for k, v in extra.items():
        if v is None:
            g.pop(k, None)
        else:
            g[k] = v.detach().float().cpu()
    pb = O.Problem(case["cam"], g, bg=bg, quick=quick)
    return pb, O.forward(pb)


@pytest.mark.parametrize("variant", ["rgb", "rgb_cov_python", "rgb_sh_python", "rgb_white_bg"])
def test_render_pattern_rgb_modes(gpu, oracle_lib, variant):
    case, pc, cam = _setup("rgb", gpu)
    pipe = SimpleNamespace(debug=False, compute_cov3D_python=variant == "rgb_cov_python",
                           convert_SHs_python=variant == "rgb_sh_python")
    opt = SimpleNamespace(include_feature=False, quick_render=False, topk=4)
    bgv = (1.0, 1.0, 1.0) if variant == "rgb_white_bg" else (0.0, 0.0, 0.0)
    out = render_like_reference(cam, pc, pipe, torch.tensor(bgv, device=gpu), opt)
    if out["_colors"] is not None:
        out["_colors"].retain_grad()
    if out["_cov"] is not None:
        out["_cov"].retain_grad()
    assert out["language_feature_weight_map"].shape == (0, 96, 112)
    extra = {}
    if out["_colors"] is not None:
        extra.update(colors_precomp=out["_colors"], shs=None)
    if out["_cov"] is not None:
        extra.update(cov3D_precomp=out["_cov"], scales=None, rotations=None)
    pb, ref = _oracle(case, pc, extra, bg=bgv)
    np.testing.assert_array_equal(out["render"].detach().cpu().numpy(), ref["color"])
    np.testing.assert_array_equal(out["radii"].cpu().numpy(), ref["radii"])
    assert torch.equal(out["visibility_filter"].cpu(), torch.from_numpy(ref["radii"] > 0))
    dC = np.random.default_rng(2).standard_normal((3, 96, 112)).astype(np.float32)
    out["render"].backward(torch.from_numpy(dC).to(gpu))
    rb = oracle_lib.backward(pb, ref, dC, None)
    # means2D is the non-leaf `zeros_like + 0`: its gradient arrives through retain_grad
    m2d = out["viewspace_points"].grad
    assert m2d is not None and not bool(m2d[:, 2].any())
    assert_grad_close("means2D", m2d.cpu().numpy(), rb["dmean2D"])
    assert_grad_close("opacity", pc.opacity.grad.cpu().numpy(), rb["dopacity"][:, None])
    if out["_colors"] is not None:
        assert_grad_close("colors_precomp", out["_colors"].grad.cpu().numpy(), rb["dcolors"])
        assert pc.features.grad is not None and bool(torch.isfinite(pc.features.grad).all())
    else:
        assert_grad_close("features", pc.features.grad.cpu().numpy(), rb["dsh"])
    if out["_cov"] is not None:
        assert_grad_close("cov3D", out["_cov"].grad.cpu().numpy(), rb["dcov3D"])
        assert pc.scaling.grad is not None and bool(torch.isfinite(pc.scaling.grad).all())
    else:
        assert_grad_close("scaling", pc.scaling.grad.cpu().numpy(), rb["dscales"])
        assert_grad_close("rotation", pc.rotation.grad.cpu().numpy(), rb["drot"])
    if out["_colors"] is None:
        assert_grad_close("xyz", pc.xyz.grad.cpu().numpy(), rb["dmeans3D"])
    # train.py:247-251: the densification bookkeeping the outputs feed
    vis = out["visibility_filter"]
    max_r = torch.zeros(pc.xyz.shape[0], device=gpu)
    max_r[vis] = torch.max(max_r[vis], out["radii"][vis])
    grad_acc = torch.norm(m2d[vis, :2], dim=-1, keepdim=True)
    assert bool((max_r[vis] > 0).all()) and bool(torch.isfinite(grad_acc).all())


def test_render_pattern_feature_mode(gpu, oracle_lib):
    case, pc, cam = _setup("feature", gpu)
    pipe = SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=False)
    opt = SimpleNamespace(include_feature=True, quick_render=False, topk=4)
    out = render_like_reference(cam, pc, pipe, torch.zeros(3, device=gpu), opt)
    lw = out["_lw"]
    lw.retain_grad()
    assert out["language_feature_weight_map"].shape == (64, 96, 112)
    pb, ref = _oracle(case, pc, {"language_feature_precomp": lw})
    # 64 dense language channels: the fast-exp ML form (harness.FWD_ATOL_FX)
    assert_img(out["render"].detach().cpu().numpy(), ref["color"], FWD_ATOL_FX, "color")
    assert_img(out["language_feature_weight_map"].detach().cpu().numpy(), ref["lang"], FWD_ATOL_FX, "lang")
    rng = np.random.default_rng(3)
    dC = rng.standard_normal((3, 96, 112)).astype(np.float32)
    dL = rng.standard_normal((64, 96, 112)).astype(np.float32)
    torch.autograd.backward([out["render"], out["language_feature_weight_map"]],
                            [torch.from_numpy(dC).to(gpu), torch.from_numpy(dL).to(gpu)])
    rb = oracle_lib.backward(pb, ref, dC, dL)
    assert_grad_close("codes", lw.grad.cpu().numpy(), rb["dlang"])
    assert_grad_close("means2D", out["viewspace_points"].grad.cpu().numpy(), rb["dmean2D"])
    assert pc.logits.grad is not None and bool(torch.isfinite(pc.logits.grad).all())


def test_render_pattern_quick_mode_with_include_feature(gpu, oracle_lib):
    """eval_lerf.sh sets include_feature AND quick_render: the forward renders the 192
    quick channels, and a backward of the RGB image (geometry gradients) must run."""
    case, pc, cam = _setup("quick", gpu)
    pipe = SimpleNamespace(debug=False, compute_cov3D_python=False, convert_SHs_python=False)
    opt = SimpleNamespace(include_feature=True, quick_render=True, topk=4)
    out = render_like_reference(cam, pc, pipe, torch.zeros(3, device=gpu), opt)
    assert out["language_feature_weight_map"].shape == (192, 96, 112)
    pb, ref = _oracle(case, pc, {}, quick=True)
    np.testing.assert_array_equal(out["render"].detach().cpu().numpy(), ref["color"])
    np.testing.assert_array_equal(out["language_feature_weight_map"].detach().cpu().numpy(), ref["lang"])
    dC = np.random.default_rng(4).standard_normal((3, 96, 112)).astype(np.float32)
    out["render"].backward(torch.from_numpy(dC).to(gpu))
    rb = oracle_lib.backward(pb, ref, dC, None)
    assert_grad_close("means2D", out["viewspace_points"].grad.cpu().numpy(), rb["dmean2D"])
    assert_grad_close("xyz", pc.xyz.grad.cpu().numpy(), rb["dmeans3D"])
    assert_grad_close("features", pc.features.grad.cpu().numpy(), rb["dsh"])
    assert_grad_close("opacity", pc.opacity.grad.cpu().numpy(), rb["dopacity"][:, None])

