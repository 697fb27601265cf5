"""Fused top-k soft-code producer (csrc/lang_codes.hip)
against the reference's own outputs (tests/golden/ref_utils.npz, made by
tests/golden/make_ref_golden.py from utils/vq_utils.py) and against the
float64 oracle restatement (oracle/oracle.py) at larger sizes.

Tolerances: codes are fp32 softmax values renormalised over k entries:
CODE_ATOL = 1e-6 absolute (values lie in [0, 1]).  Gradients: GRAD_RTOL =
2e-6 relative to max(1, max|ref|).  The selected channels (mask, indices)
are compared exactly, except where the oracle's k-th and (k+1)-th softmax
values lie within 1e-6 relative (an fp32 near-tie, where either choice is
the reference's; torch.topk's own tie order is implementation-defined).
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_utils.npz"))
CODE_ATOL = 1e-6
GRAD_RTOL = 2e-6

pytestmark = pytest.mark.gpu


def _lc():
    from langsplatv2_amd import lang_codes
    return lang_codes


def _near_tie_rows(x: np.ndarray, k: int, levels: int) -> np.ndarray:
    """Rows where some level's k-th and (k+1)-th softmax values are within 1e-6 relative."""
    N, LK = x.shape
    K = LK // levels
    bad = np.zeros(N, bool)
    if k >= K:
        return bad
    for l in range(levels):
        y = np.sort(O._softmax(x[:, l * K:(l + 1) * K].astype(np.float64)), axis=1)[:, ::-1]
        bad |= (y[:, k - 1] - y[:, k]) <= 1e-6 * y[:, k - 1]
    return bad


@pytest.mark.parametrize("k", [1, 4, 8])
def test_dense_codes_match_reference(gpu, k):
    x = torch.from_numpy(G["lang_logits"]).to(gpu)
    out = _lc().softmax_to_topk_soft_code(x, k).cpu().numpy()
    np.testing.assert_allclose(out, G[f"lang_topk{k}"], rtol=0, atol=CODE_ATOL)
    np.testing.assert_array_equal(out != 0, G[f"lang_topk{k}"] != 0)


def test_sparse_codes_match_reference(gpu):
    x = torch.from_numpy(G["lang_logits"]).to(gpu)
    w, idx = _lc().get_weights_and_indices(x, 4)
    assert w.dtype == torch.float32 and idx.dtype == torch.float32
    np.testing.assert_allclose(w.cpu().numpy(), G["lang_quick_w"], rtol=0, atol=CODE_ATOL)
    np.testing.assert_array_equal(idx.cpu().numpy(), G["lang_quick_idx"])


def test_grad_matches_reference_autograd(gpu):
    x = torch.from_numpy(G["lang_logits"]).to(gpu).requires_grad_(True)
    code = _lc().softmax_to_topk_soft_code(x, 4)
    (dx,) = torch.autograd.grad(code, x, torch.from_numpy(G["lang_grad_up"]).to(gpu))
    ref = G["lang_topk4_dlogits"]
    np.testing.assert_allclose(dx.cpu().numpy(), ref, rtol=0, atol=GRAD_RTOL * max(1.0, np.abs(ref).max()))


def test_multilevel_matches_reference(gpu):
    x = torch.from_numpy(G["lang3_logits"]).to(gpu)
    lc = _lc()
    dense = lc.get_render_weights(x, 3, 64, 4).cpu().numpy()
    np.testing.assert_allclose(dense, G["lang3_render_weights"], rtol=0, atol=CODE_ATOL)
    w, idx = lc.quick_inputs(x, 4, levels=3)
    np.testing.assert_allclose(w.cpu().numpy(), G["lang3_quick_w"], rtol=0, atol=CODE_ATOL)
    np.testing.assert_array_equal(idx.cpu().numpy(), G["lang3_quick_idx"])


@pytest.mark.parametrize("K,k,levels", [(64, 4, 1), (64, 1, 3), (128, 16, 1), (192, 4, 2), (256, 8, 1), (64, 64, 1)])
def test_random_rows_match_oracle(gpu, K, k, levels):
    gen = torch.Generator().manual_seed(K * 1000 + k * 10 + levels)
    N = 20000
    x = (torch.randn(N, levels * K, generator=gen) * 2.0)
    xn = x.numpy()
    lc = _lc()
    xd = x.to(gpu).requires_grad_(True)
    code = lc.get_render_weights(xd, levels, K, k)
    ok = ~_near_tie_rows(xn, k, levels)
    assert ok.sum() > 0.99 * N
    ref = O.topk_soft_code(xn, k, levels)
    got = code.detach().cpu().numpy()
    np.testing.assert_array_equal((got != 0)[ok], (ref != 0)[ok])
    np.testing.assert_allclose(got[ok], ref[ok], rtol=0, atol=CODE_ATOL)
    # backward
    gup = torch.randn(N, levels * K, generator=gen)
    (dx,) = torch.autograd.grad(code, xd, gup.to(gpu))
    dref = O.topk_soft_code_backward(xn, gup.numpy(), k, levels)
    np.testing.assert_allclose(dx.cpu().numpy()[ok], dref[ok], rtol=0,
                               atol=GRAD_RTOL * max(1.0, np.abs(dref).max()))
    # sparse form, every index dtype
    wref, iref = O.weights_and_indices(xn, k, levels)
    for dt in (torch.float32, torch.int32, torch.int64):
        w, idx = lc.quick_inputs(xd.detach(), k, levels=levels, index_dtype=dt)
        assert idx.dtype == dt
        np.testing.assert_array_equal(idx.cpu().numpy().astype(np.int64)[ok], iref[ok])
        np.testing.assert_allclose(w.cpu().numpy()[ok], wref[ok], rtol=0, atol=CODE_ATOL)


def test_ties_take_the_lower_channel_and_edges(gpu):
    lc = _lc()
    x = torch.zeros(3, 64)
    x[1, [10, 20, 30]] = 1.0          # 3 clear winners + 61-way tie for the 4th slot
    x[2] = torch.arange(64).float()   # strictly increasing
    w, idx = lc.quick_inputs(x.to(gpu), 4, index_dtype=torch.int64)
    idx = idx.cpu().numpy()
    np.testing.assert_array_equal(idx[0], [0, 1, 2, 3])
    np.testing.assert_array_equal(idx[1], [0, 10, 20, 30])
    np.testing.assert_array_equal(idx[2], [60, 61, 62, 63])
    np.testing.assert_allclose(w.cpu().numpy()[0], np.full(4, 0.25), atol=1e-7)
    # N = 0
    e = lc.softmax_to_topk_soft_code(torch.zeros(0, 64, device=gpu), 4)
    assert e.shape == (0, 64)
    # unsupported codebook width and CPU tensors fail loudly
    with pytest.raises(RuntimeError):
        lc.softmax_to_topk_soft_code(torch.zeros(4, 48, device=gpu), 4)
    with pytest.raises(RuntimeError):
        lc.softmax_to_topk_soft_code(torch.zeros(4, 64), 4)


def test_codes_feed_the_rasterizer_quick_path(gpu):
    """quick_inputs -> the rasterizer's sparse language input: the rendered
    64-channel map equals a render of the dense codes of the same logits."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from langsplatv2_amd import scenes
    cam = scenes.make_camera(64, 48)
    g = scenes.make_gaussians(800, cam, seed=3, sh_degree=None)
    gen = torch.Generator().manual_seed(7)
    logits = torch.randn(800, 64, generator=gen).to(gpu)
    lc = _lc()
    w, idx = lc.quick_inputs(logits, 4)
    dense = lc.softmax_to_topk_soft_code(logits, 4)
    dev = {k: (v.to(gpu) if isinstance(v, torch.Tensor) else v) for k, v in g.items()}

    def rs(quick):
        return GaussianRasterizationSettings(
            image_height=48, image_width=64, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
            bg=torch.zeros(3, device=gpu), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(gpu),
            projmatrix=cam["projmatrix"].to(gpu), sh_degree=0, campos=cam["campos"].to(gpu), prefiltered=False,
            debug=False, include_feature=True, quick_render=quick, language_feature_dim=64 if quick else None)

    common = dict(means3D=dev["means3D"], means2D=torch.zeros_like(dev["means3D"]), opacities=dev["opacities"],
                  colors_precomp=dev["colors_precomp"], scales=dev["scales"], rotations=dev["rotations"])
    with torch.no_grad():
        _, lq, _ = GaussianRasterizer(rs(True))(language_feature_weights_quick=w, language_feature_indices=idx,
                                                 **common)
        _, ld, _ = GaussianRasterizer(rs(False))(language_feature_precomp=dense, **common)
    assert lq.shape == ld.shape == (64, 48, 64)
    np.testing.assert_allclose(lq.cpu().numpy(), ld.cpu().numpy(), rtol=0, atol=2e-6)
