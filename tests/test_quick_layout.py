"""The quick map's pixel-major layout (language_feature_layout="hwc",
lsr_settings.quick_layout = LSR_LAYOUT_HWC; the default whenever the 12-code,
192-channel kernel applies) and the decode reading it.

The reference returns the quick weight map as a contiguous (192, H, W) tensor
(gaussian_renderer/__init__.py:108-129) and its consumers reshape it with
.view(3, 64, H, W).view(3, 64, H*W) before the einsum (eval_lerf.py:214-217,
backend_renderer.py:24-31).  The "hwc" layout stores each pixel's 192 weights
contiguously and returns the (192, H, W) view with strides (1, 192 W, 192):
the same values (bit-exact against the oracle and against the reference
layout), and those .view calls and the einsum run on it unchanged.  The decode
(csrc/quick.hip, k_quick_decode_l<., ., HWC>) reads it in 32-B pieces; its
arithmetic is the same, so its output equals the reference-layout decode bit
for bit."""
import numpy as np
import pytest
import torch

from harness import assert_img, make_case, oracle_problem, settings_for

QUICK = dict(N=5000, W=128, H=96, sh_degree=None, quick_k=4, seed=9)


def test_layout_setting_validation():
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    from langsplatv2_amd import _lib, rasterizer
    base = dict(image_height=8, image_width=8, tanfovx=0.5, tanfovy=0.5, bg=torch.zeros(3), scale_modifier=1.0,
                viewmatrix=torch.eye(4), projmatrix=torch.eye(4), sh_degree=0, campos=torch.zeros(3),
                prefiltered=False, debug=False)
    assert rasterizer._quick_layout(GaussianRasterizationSettings(**base)) == _lib.LSR_LAYOUT_CHW
    # the default (None): pixel-major for a quick render whose inputs fit its kernel, else channel-major
    assert rasterizer._quick_layout(GaussianRasterizationSettings(**base, quick_render=True), True) == _lib.LSR_LAYOUT_HWC
    assert rasterizer._quick_layout(GaussianRasterizationSettings(**base, quick_render=True), False) == _lib.LSR_LAYOUT_CHW
    assert rasterizer._quick_layout(GaussianRasterizationSettings(**base), True) == _lib.LSR_LAYOUT_CHW
    assert rasterizer._quick_layout(GaussianRasterizationSettings(**base, quick_render=True,
                                                                  language_feature_layout="chw"), True) == _lib.LSR_LAYOUT_CHW
    assert rasterizer._quick_layout(GaussianRasterizationSettings(**base, quick_render=True,
                                                                  language_feature_layout="hwc")) == _lib.LSR_LAYOUT_HWC
    with pytest.raises(ValueError, match="quick_render map only"):
        rasterizer._quick_layout(GaussianRasterizationSettings(**base, language_feature_layout="hwc"))
    with pytest.raises(ValueError, match="must be"):
        rasterizer._quick_layout(GaussianRasterizationSettings(**base, quick_render=True, language_feature_layout="nhwc"))


def _render_quick(case, gpu, layout):
    from diff_gaussian_rasterization import GaussianRasterizer
    t = {k: v.to(gpu) for k, v in case["g"].items() if isinstance(v, torch.Tensor)}
    r = GaussianRasterizer(raster_settings=settings_for(case, gpu, layout))
    kw = {k: t[k] for k in ("shs", "colors_precomp", "scales", "rotations") if k in t}
    with torch.no_grad():
        color, lang, radii = r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                               language_feature_weights_quick=t["language_feature_weights_quick"],
                               language_feature_indices=t["language_feature_indices"], **kw)
    return color, lang, radii


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(128, 96), (45, 37)])
def test_hwc_map_equals_reference_layout_and_oracle(gpu, W, H):
    from oracle import oracle as O
    case = make_case(**dict(QUICK, W=W, H=H))
    c0, m0, r0 = _render_quick(case, gpu, "chw")
    c1, m1, r1 = _render_quick(case, gpu, "hwc")
    assert m0.is_contiguous() and m1.shape == m0.shape == (192, H, W)
    assert m1.stride() == (1, 192 * W, 192)
    assert torch.equal(m1, m0) and torch.equal(c1, c0) and torch.equal(r1, r0)
    ref = O.forward(oracle_problem(case))
    assert_img(m1.cpu().numpy(), ref["lang"], 0.0, "lang (hwc)")
    # the reference consumers' reshapes and einsum (eval_lerf.py:214-217) on the hwc view
    cb = torch.randn(3, 64, 512, generator=torch.Generator().manual_seed(3)).to(gpu)
    e0 = torch.einsum("ldk,lkn->ldn", cb.permute(0, 2, 1), m0.view(3, 64, H, W).view(3, 64, H * W))
    e1 = torch.einsum("ldk,lkn->ldn", cb.permute(0, 2, 1), m1.view(3, 64, H, W).view(3, 64, H * W))
    torch.testing.assert_close(e1, e0, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_hwc_decode_bit_exact_with_reference_layout(gpu):
    from langsplatv2_amd import quick
    from test_quick_decode import DEC_ATOL, ref_decode
    case = make_case(**QUICK)
    _, m0, _ = _render_quick(case, gpu, "chw")
    _, m1, _ = _render_quick(case, gpu, "hwc")
    cb = torch.randn(3, 64, 512, generator=torch.Generator().manual_seed(4)).to(gpu)
    for normalize in (False, True):
        d0 = quick.decode_language_features(m0, cb, normalize=normalize)
        d1 = quick.decode_language_features(m1, cb, normalize=normalize)
        assert d1.is_contiguous() and torch.equal(d1, d0)
    np.testing.assert_allclose(d1.cpu().numpy(), ref_decode(m0.cpu().numpy(), cb.cpu().numpy()), atol=DEC_ATOL, rtol=0)


@pytest.mark.gpu
def test_hwc_decode_synthetic_ragged(gpu):
    """A pixel-major map built directly (ragged width, sparse weights) decodes as
    its contiguous copy does."""
    from langsplatv2_amd import quick
    g = torch.Generator().manual_seed(5)
    H, W = 29, 83
    hwc = (torch.rand(H, W, 192, generator=g) * (torch.rand(H, W, 192, generator=g) < 0.15)).to(gpu)
    m = hwc.permute(2, 0, 1)
    cb = torch.randn(3, 64, 512, generator=g).to(gpu)
    assert torch.equal(quick.decode_language_features(m, cb), quick.decode_language_features(m.contiguous(), cb))


@pytest.mark.gpu
def test_hwc_unsupported_shapes_raise(gpu):
    """The pixel-major map is written by the 12-code, 192-channel kernel only:
    asked for explicitly on other inputs it raises, and the default falls back
    to the reference's contiguous map."""
    case = make_case(**dict(QUICK, quick_k=2))   # 3 levels x top-2 = 6 codes
    with pytest.raises(RuntimeError):
        _render_quick(case, gpu, "hwc")
    _, m_def, _ = _render_quick(case, gpu, None)
    _, m_chw, _ = _render_quick(case, gpu, "chw")
    assert m_def.is_contiguous() and torch.equal(m_def, m_chw)


def _consumers(m, cb, H, W):
    """The reference's consumer patterns of the quick weight map, verbatim in shape:
    eval_lerf.py:213-218 (eval_3d_ovs.py:279-283, eval_mip_nerf360.py:171-175,
    demo_prompt.py:24-36 and backend_renderer.py / debug_renderer.py:19-33 are the
    same .view + einsum + norm), and compute_final_feature_map's .view(D, -1) matmul
    (scene/gaussian_model.py:545-550; layer / per-level slices :520-543)."""
    out = {}
    D, h, w = m.shape
    wm = m.view(3, 64, h, w).view(3, 64, h * w)
    f = torch.einsum("ldk,lkn->ldn", cb.permute(0, 2, 1), wm).view(3, 512, h, w)
    out["einsum"] = f
    out["einsum_norm"] = f / (f.norm(dim=1, keepdim=True) + 1e-10)
    flat = m.view(D, -1)
    out["final"] = (cb.reshape(-1, 512).T @ flat).view(512, h, w)
    out["levels"] = torch.stack([cb[i].T @ flat[i * 64:(i + 1) * 64] for i in range(3)])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(128, 96), (45, 37)])
def test_default_layout_serves_every_reference_consumer(gpu, W, H):
    """With default settings (no language_feature_layout) the quick map is the
    pixel-major view, and every consumer pattern of the reference gives the
    same result on it as on the reference's contiguous map."""
    case = make_case(**dict(QUICK, W=W, H=H))
    _, m_def, _ = _render_quick(case, gpu, None)
    _, m_chw, _ = _render_quick(case, gpu, "chw")
    assert m_def.stride() == (1, 192 * W, 192) and m_chw.is_contiguous()
    assert torch.equal(m_def, m_chw)
    cb = torch.randn(3, 64, 512, generator=torch.Generator().manual_seed(11)).to(gpu)
    a, b = _consumers(m_def, cb, H, W), _consumers(m_chw, cb, H, W)
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-5, msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
def test_hwc_integer_indices(gpu, idx_dtype):
    """The pixel-major map with int32 / int64 code indices (u5: the integer
    index forms of language_feature_indices) equals the fp32-index map."""
    from diff_gaussian_rasterization import GaussianRasterizer
    case = make_case(**dict(QUICK, W=61, H=47))
    t = {k: v.to(gpu) for k, v in case["g"].items() if isinstance(v, torch.Tensor)}
    r = GaussianRasterizer(raster_settings=settings_for(case, gpu, "hwc"))
    kw = {k: t[k] for k in ("shs", "colors_precomp", "scales", "rotations") if k in t}
    outs = []
    for qi in (t["language_feature_indices"], t["language_feature_indices"].round().to(idx_dtype)):
        with torch.no_grad():
            _, lang, _ = r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                           language_feature_weights_quick=t["language_feature_weights_quick"],
                           language_feature_indices=qi.contiguous(), **kw)
        outs.append(lang)
    assert outs[1].stride() == (1, 192 * 61, 192)
    assert torch.equal(outs[0], outs[1])
