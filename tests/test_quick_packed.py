"""Packed quick code rows (LSR_INDEX_PACKED, lsr_quick_pack_codes).

The reference hands the rasterizer its quick code indices as an (N, 12) fp32
tensor (eval_lerf.py:340-348, gaussian_renderer/__init__.py:87-93), and the
quick render reads 12 of them per staged candidate.  The forward converts that
tensor once into 16-B rows of code + 1 bytes (rasterizer._packed_codes, kept
while the tensor is unchanged) and the render stages the rows as they are.
Same codes, same render: the outputs equal the unpacked path bit for bit."""
import numpy as np
import pytest
import torch

from harness import make_case, settings_for

QUICK = dict(N=5000, W=128, H=96, sh_degree=None, quick_k=4, seed=9)


def test_packed_constants_and_export():
    from langsplatv2_amd import _lib
    assert _lib.LSR_INDEX_PACKED == 3
    assert "lsr_quick_pack_codes" in _lib.EXPORTS


def _ref_pack(idx: np.ndarray, Dq: int) -> np.ndarray:
    """Restatement of the pack: fp32 codes round half up (u5), int codes as
    they are; code + 1 when 0 <= code < Dq, else 0; byte m of row i."""
    if idx.dtype == np.float32:
        q = np.floor(idx + np.float32(0.5)).astype(np.float64)   # the fp32 sum, as the kernel forms it
    else:
        q = idx.astype(np.float64)
    b = np.where((q >= 0) & (q < Dq), q + 1, 0).astype(np.uint32)
    w = np.zeros((idx.shape[0], 4), dtype=np.uint32)
    for m in range(12):
        w[:, m // 4] |= b[:, m] << np.uint32(8 * (m % 4))
    return w.view(np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.int32, torch.int64])
def test_pack_codes_match_restatement(gpu, dtype):
    from langsplatv2_amd import rasterizer
    g = torch.Generator().manual_seed(3)
    N = 4099
    if dtype == torch.float32:
        idx = torch.randint(-3, 200, (N, 12), generator=g).float() + (torch.rand(N, 12, generator=g) - 0.5) * 0.98
        idx[0, :6] = torch.tensor([191.5, 191.49, -0.5, -0.51, 1e10, -1e10])
    else:
        idx = torch.randint(-3, 200, (N, 12), generator=g).to(dtype)
        if dtype == torch.int64:
            idx[0, :3] = torch.tensor([2 ** 32 + 5, -(2 ** 40), 2 ** 31])
    for Dq in (192, 64):
        rasterizer._PACKED.clear()
        got = rasterizer._packed_codes(idx.to(gpu).contiguous(), Dq).cpu().numpy()
        np.testing.assert_array_equal(got, _ref_pack(idx.numpy(), Dq))


def test_pack_codes_rejects_bad_arguments():
    from langsplatv2_amd import _lib
    lib = _lib.load()
    assert lib.lsr_quick_pack_codes(None, _lib.LSR_INDEX_F32, 0, 12, 192, None, None) == _lib.LSR_OK
    assert lib.lsr_quick_pack_codes(None, _lib.LSR_INDEX_F32, 0, 8, 192, None, None) == 2        # K != 12
    assert lib.lsr_quick_pack_codes(None, _lib.LSR_INDEX_PACKED, 0, 12, 192, None, None) == 1    # not a source
    assert lib.lsr_quick_pack_codes(None, _lib.LSR_INDEX_F32, 0, 12, 256, None, None) == 2       # byte codes


def _render(case, gpu, layout=None, qi=None, packed=True, w=None):
    from diff_gaussian_rasterization import GaussianRasterizer
    from langsplatv2_amd import rasterizer
    t = {k: v.to(gpu) for k, v in case["g"].items() if isinstance(v, torch.Tensor)}
    r = GaussianRasterizer(raster_settings=settings_for(case, gpu, layout))
    kw = {k: t[k] for k in ("shs", "colors_precomp", "scales", "rotations") if k in t}
    old = rasterizer.QUICK_PACKED_CODES
    rasterizer.QUICK_PACKED_CODES = packed
    try:
        with torch.no_grad():
            return r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                     language_feature_weights_quick=t["language_feature_weights_quick"] if w is None else w,
                     language_feature_indices=t["language_feature_indices"] if qi is None else qi, **kw)
    finally:
        rasterizer.QUICK_PACKED_CODES = old


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["chw", None])
@pytest.mark.parametrize("W,H", [(128, 96), (45, 37)])
def test_packed_render_equals_index_render(gpu, layout, W, H):
    from langsplatv2_amd import rasterizer
    case = make_case(**dict(QUICK, W=W, H=H))
    qi = case["g"]["language_feature_indices"].to(gpu)
    rasterizer._PACKED.clear()
    c0, m0, r0 = _render(case, gpu, layout, qi, packed=False)
    c1, m1, r1 = _render(case, gpu, layout, qi, packed=True)
    assert len(rasterizer._PACKED) == 1   # the packed rows were used (and kept)
    assert torch.equal(m1, m0) and torch.equal(c1, c0) and torch.equal(r1, r0)
    for dt in (torch.int32, torch.int64):
        c2, m2, _ = _render(case, gpu, layout, qi.round().to(dt).contiguous(), packed=True)
        assert torch.equal(m2, m0) and torch.equal(c2, c0)


@pytest.mark.gpu
def test_packed_rows_follow_in_place_changes(gpu):
    """The kept rows are reused only while the indices tensor is unchanged: an
    in-place edit bumps its version counter and the next forward re-packs."""
    from langsplatv2_amd import rasterizer
    case = make_case(**QUICK)
    qi = case["g"]["language_feature_indices"].to(gpu).clone()
    rasterizer._PACKED.clear()
    _render(case, gpu, None, qi)
    first = next(iter(rasterizer._PACKED.values()))[2]
    _, m_again, _ = _render(case, gpu, None, qi)
    assert next(iter(rasterizer._PACKED.values()))[2] is first        # reused
    qi[:, :4] = torch.remainder(qi[:, :4] + 17.0, 64.0)                 # new level-0 codes
    _, m1, _ = _render(case, gpu, None, qi)
    _, m0, _ = _render(case, gpu, None, qi, packed=False)
    assert torch.equal(m1, m0) and not torch.equal(m1, m_again)
    assert len(rasterizer._PACKED) <= rasterizer._PACKED_MAX


@pytest.mark.gpu
def test_packed_cache_holds_no_indices_tensor(gpu):
    """a cache entry references its indices tensor weakly, so a tensor
    the caller drops is freed (and its packed rows can never be reused for
    another tensor that lands in the same storage)."""
    import gc
    import weakref
    from langsplatv2_amd import rasterizer
    case = make_case(**QUICK)
    qi = case["g"]["language_feature_indices"].to(gpu).clone()
    rasterizer._PACKED.clear()
    _render(case, gpu, None, qi)
    w = weakref.ref(qi)
    del qi
    gc.collect()
    assert w() is None
    assert len(rasterizer._PACKED) == 1 and next(iter(rasterizer._PACKED.values()))[0]() is None
    qi2 = case["g"]["language_feature_indices"].to(gpu).clone()
    _, m2, _ = _render(case, gpu, None, qi2)
    _, m0, _ = _render(case, gpu, None, qi2, packed=False)
    assert torch.equal(m2, m0)


@pytest.mark.gpu
def test_packed_bytes_above_dq_are_dropped(gpu, monkeypatch):
    """Hand-made rows with bytes above Dq render as those codes out of range
    (the render never indexes past its Dq accumulators)."""
    from langsplatv2_amd import rasterizer
    case = make_case(**QUICK)
    qi = case["g"]["language_feature_indices"].to(gpu)
    rasterizer._PACKED.clear()
    packed = rasterizer._packed_codes(qi, 192).clone()
    b = packed.view(torch.uint8).view(-1, 16)
    b[::3, 1] = 250          # code 1 of every third Gaussian
    b[1::5, 9] = 193         # code 9 of every fifth, from the second
    monkeypatch.setattr(rasterizer, "_packed_codes", lambda t, Dq: packed)
    c1, m1, _ = _render(case, gpu, None, qi)
    ref = qi.clone()
    ref[::3, 1] = -1.0
    ref[1::5, 9] = 1000.0
    c0, m0, _ = _render(case, gpu, None, ref, packed=False)
    assert torch.equal(m1, m0) and torch.equal(c1, c0)


@pytest.mark.gpu
def test_packed_forward_keeps_quick_weight_gradient(gpu):
    """The quick weights' gradient after a packed forward
    equals the one after an unpacked forward (the backward reads the caller's
    indices either way).  The quick backward takes Dq <= 64: the 12 codes are
    folded into 64 channels."""
    case = make_case(**QUICK)
    case["g"]["quick_dim"] = 64
    case["g"]["language_feature_indices"] = torch.remainder(case["g"]["language_feature_indices"], 64.0)
    t = {k: v.to(gpu) for k, v in case["g"].items() if isinstance(v, torch.Tensor)}
    from diff_gaussian_rasterization import GaussianRasterizer
    from langsplatv2_amd import rasterizer
    r = GaussianRasterizer(raster_settings=settings_for(case, gpu))
    dl = torch.randn(64, QUICK["H"], QUICK["W"], generator=torch.Generator().manual_seed(2)).to(gpu)
    grads = []
    for packed in (False, True):
        rasterizer.QUICK_PACKED_CODES = packed
        try:
            w = t["language_feature_weights_quick"].clone().requires_grad_(True)
            _, lang, _ = r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                           colors_precomp=t["colors_precomp"], scales=t["scales"], rotations=t["rotations"],
                           language_feature_weights_quick=w, language_feature_indices=t["language_feature_indices"])
            (g,) = torch.autograd.grad(lang, w, dl)
            grads.append(g)
        finally:
            rasterizer.QUICK_PACKED_CODES = True
    torch.testing.assert_close(grads[1], grads[0], rtol=1e-6, atol=1e-6 * float(grads[0].abs().max()))
