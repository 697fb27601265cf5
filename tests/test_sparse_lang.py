"""The sparse (N, k) language input WITH a gradient through the rasterizer
(SURVEY §8f rank 2): the fused top-k producer's packed codes (weights, codes)
rendered with quick_render=True into Dq channels, dL/dweights from the
backward, dL/dlogits from the producer's sparse backward — so feature-mode
training never forms the dense (N, 64) codes of get_render_weights
(scene/gaussian_model.py:510-518, utils/vq_utils.py:9-24).

Parity:
  * forward (quick, Dq = 64) bit-exact vs the oracle;
  * dL/dweights (language-only backward, the training path) vs the oracle's
    sparse backward (dense expansion + gather, oracle/oracle.py) within
    tests/harness.py's GRAD_RTOL;
  * sparse == dense: the same codes rendered densely (include_feature, D = 64)
    give dL/dcode gathered at the codes == dL/dweights, and the same dL/dlogits;
  * geometry + sparse language gradients together (expansion path) vs oracle.
"""
import numpy as np
import pytest
import torch

from harness import assert_grad_close, make_case

N, W, H = 4000, 128, 96


def _setup(dev, seed=21, index_dtype=torch.int32):
    from langsplatv2_amd import lang_codes
    case = make_case(N=N, W=W, H=H, sh_degree=3, seed=seed)
    logits = torch.randn(N, 64, generator=torch.Generator().manual_seed(seed)).to(dev).requires_grad_(True)
    w, idx = lang_codes.sparse_codes(logits, 4, levels=1, index_dtype=index_dtype)
    return case, logits, w, idx


def _settings(case, dev, quick, include_feature, qdim=64):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    cam = case["cam"]
    return GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"], bg=torch.zeros(3, device=dev),
        scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev), projmatrix=cam["projmatrix"].to(dev), sh_degree=3,
        campos=cam["campos"].to(dev), prefiltered=False, debug=False, include_feature=include_feature,
        quick_render=quick, language_feature_dim=qdim if quick else None)


def _geom(case, dev, grad=False):
    return {k: case["g"][k].to(dev).clone().requires_grad_(grad)
            for k in ("means3D", "shs", "opacities", "scales", "rotations")}


def _oracle(case, w, idx, quick=True):
    from oracle import oracle as O
    g = dict(case["g"])
    g["language_feature_weights_quick"] = w.detach().cpu()
    g["language_feature_indices"] = idx.detach().cpu().float()
    g["quick_dim"] = 64
    pb = O.Problem(case["cam"], g, quick=quick)
    return pb, O.forward(pb)


def _dl(seed=5):
    return np.random.default_rng(seed).standard_normal((64, H, W)).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("index_dtype", [torch.int32, torch.float32, torch.int64])
def test_sparse_language_only_backward_vs_oracle(gpu, oracle_lib, index_dtype):
    from diff_gaussian_rasterization import GaussianRasterizer
    case, logits, w, idx = _setup(gpu, index_dtype=index_dtype)
    assert w.requires_grad and not idx.requires_grad and w.shape == (N, 4)
    t = _geom(case, gpu)
    r = GaussianRasterizer(_settings(case, gpu, True, True))
    color, lmap, radii = r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                           shs=t["shs"], language_feature_weights_quick=w, language_feature_indices=idx,
                           scales=t["scales"], rotations=t["rotations"])
    w.retain_grad()
    pb, ref = _oracle(case, w, idx)
    np.testing.assert_array_equal(lmap.detach().cpu().numpy(), ref["lang"])
    np.testing.assert_array_equal(color.detach().cpu().numpy(), ref["color"])
    dL = _dl()
    lmap.backward(torch.from_numpy(dL).to(gpu))
    rb = oracle_lib.backward(pb, ref, np.zeros((3, H, W), np.float32), dL)
    assert_grad_close("dL/dweights", w.grad.cpu().numpy(), rb["dlang_weights"])
    assert float(np.abs(rb["dlang_weights"]).max()) > 1e-3
    assert logits.grad is not None and bool(torch.isfinite(logits.grad).all())


@pytest.mark.gpu
def test_sparse_equals_dense(gpu):
    """Same codes, two paths: quick (sparse, with grad) vs include_feature (dense (N,64))."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from langsplatv2_amd import lang_codes
    case, logits_s, w, idx = _setup(gpu)
    logits_d = logits_s.detach().clone().requires_grad_(True)
    dense = lang_codes.get_render_weights(logits_d, 1, 64, 4)
    dense.retain_grad()
    t = _geom(case, gpu)
    z = torch.zeros_like(t["means3D"])
    kw = dict(means3D=t["means3D"], means2D=z, opacities=t["opacities"], shs=t["shs"], scales=t["scales"],
              rotations=t["rotations"])
    _, ls, _ = GaussianRasterizer(_settings(case, gpu, True, True))(
        language_feature_weights_quick=w, language_feature_indices=idx, **kw)
    _, ld, _ = GaussianRasterizer(_settings(case, gpu, False, True))(language_feature_precomp=dense, **kw)
    # same codes: the packed weights are exactly the dense codes' non-zeros
    assert torch.equal(torch.gather(dense.detach(), 1, idx.long()), w.detach())
    np.testing.assert_allclose(ls.detach().cpu().numpy(), ld.detach().cpu().numpy(), rtol=0, atol=2e-7)
    w.retain_grad()
    dL = torch.from_numpy(_dl(7)).to(gpu)
    ls.backward(dL)
    ld.backward(dL)
    assert_grad_close("dL/dweights vs dense dL/dcode at the codes", w.grad.cpu().numpy(),
                      torch.gather(dense.grad, 1, idx.long()).cpu().numpy())
    assert_grad_close("dL/dlogits sparse vs dense", logits_s.grad.cpu().numpy(), logits_d.grad.cpu().numpy())


@pytest.mark.gpu
def test_sparse_language_with_geometry_vs_oracle(gpu, oracle_lib):
    """Geometry gradients AND dL/dweights in one backward (the quick channels take part
    in dL/dalpha): the library's dense-expansion path."""
    from diff_gaussian_rasterization import GaussianRasterizer
    case, logits, w, idx = _setup(gpu, seed=23)
    t = _geom(case, gpu, grad=True)
    m2d = torch.zeros_like(t["means3D"], requires_grad=True)
    r = GaussianRasterizer(_settings(case, gpu, True, True))
    color, lmap, _ = r(means3D=t["means3D"], means2D=m2d, opacities=t["opacities"], shs=t["shs"],
                       language_feature_weights_quick=w, language_feature_indices=idx, scales=t["scales"],
                       rotations=t["rotations"])
    w.retain_grad()
    pb, ref = _oracle(case, w, idx)
    rng = np.random.default_rng(9)
    dC = rng.standard_normal((3, H, W)).astype(np.float32)
    dL = rng.standard_normal((64, H, W)).astype(np.float32)
    torch.autograd.backward([color, lmap], [torch.from_numpy(dC).to(gpu), torch.from_numpy(dL).to(gpu)])
    rb = oracle_lib.backward(pb, ref, dC, dL)
    assert_grad_close("dL/dweights", w.grad.cpu().numpy(), rb["dlang_weights"])
    assert_grad_close("means2D", m2d.grad.cpu().numpy(), rb["dmean2D"])
    assert_grad_close("means3D", t["means3D"].grad.cpu().numpy(), rb["dmeans3D"])
    assert_grad_close("opacities", t["opacities"].grad.cpu().numpy(), rb["dopacity"][:, None])
    assert_grad_close("shs", t["shs"].grad.cpu().numpy(), rb["dsh"])


def test_oracle_quick_expansion_semantics(oracle_lib):
    from oracle import oracle as O
    qi = np.array([[0.49, 0.5, 63.5, 64.0], [2.0, 2.0, -1.0, 7.0]], np.float32)
    codes = O.quick_codes(qi)
    assert codes.tolist() == [[0, 1, 64, 64], [2, 2, -1, 7]]
    qw = np.array([[1.0, 2.0, 3.0, 4.0], [0.25, 0.5, 9.0, 1.0]], np.float32)
    d = O.expand_quick(qw, codes, 64)
    assert d[0, 0] == 1.0 and d[0, 1] == 2.0 and d[0].sum() == 3.0      # codes >= 64 dropped
    assert d[1, 2] == 0.75 and d[1, 7] == 1.0 and d[1].sum() == 1.75    # duplicates summed, -1 dropped


@pytest.mark.gpu
@pytest.mark.parametrize("geom_grad", [False, True])
def test_quick_weights_grad_with_colour_only_loss(gpu, oracle_lib, geom_grad):
    """Quick render whose weights require grad, with a loss on the colour only
    (autograd passes no gradient for the language map): dL/dweights is zero and
    the geometry gradients are the RGB-only ones (this used to raise
    LSR_EINVAL from the quick backward)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    case, logits, w, idx = _setup(gpu, seed=23)
    w.retain_grad()
    t = _geom(case, gpu, grad=geom_grad)
    r = GaussianRasterizer(_settings(case, gpu, True, True))
    color, lmap, _ = r(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]), opacities=t["opacities"],
                       shs=t["shs"], language_feature_weights_quick=w, language_feature_indices=idx,
                       scales=t["scales"], rotations=t["rotations"])
    dC = torch.randn(color.shape, generator=torch.Generator().manual_seed(2)).to(gpu)
    color.backward(dC)
    assert w.grad is not None and torch.count_nonzero(w.grad) == 0
    assert logits.grad is not None and torch.count_nonzero(logits.grad) == 0
    if geom_grad:
        # the same frame without the language input: identical geometry gradients
        t2 = _geom(case, gpu, grad=True)
        r2 = GaussianRasterizer(_settings(case, gpu, False, False))
        c2, _, _ = r2(means3D=t2["means3D"], means2D=torch.zeros_like(t2["means3D"]), opacities=t2["opacities"],
                      shs=t2["shs"], scales=t2["scales"], rotations=t2["rotations"])
        assert torch.equal(c2, color)
        c2.backward(dC)
        for k in ("means3D", "shs", "opacities", "scales", "rotations"):
            assert_grad_close(k, t[k].grad.cpu().numpy(), t2[k].grad.cpu().numpy())
