"""Codebook decode of the quick language map (langsplatv2_amd.quick, csrc/quick.hip)
against a float64 restatement of the reference's post-render lines
(eval_lerf.py:214-218: einsum('ldk,lkn->ldn') then / (norm + 1e-10); and
scene/gaussian_model.py:545-550 for the unnormalised dense map).

Tolerance (floating point, not bit-exact: split-f16 MFMA products with f32
accumulation, the weights scaled per pixel by a power of two before the split,
and a Cholesky-Gram norm): normalised outputs within 1e-6 absolute (values in
[-1, 1]; measured max 1.1e-7 at 1 Mpix on a rendered map and on maps scaled by
1e-3 / 1e-6, tools/dec_err.py -> profiles/r03_dec_err.json), i.e. 10x inside
the north_star's 1e-5; unnormalised within 1e-6 x max|ref|."""
import numpy as np
import pytest
import torch

from langsplatv2_amd import quick

DEC_ATOL = 1e-6


def ref_decode(wmap, cb, normalize=True, eps=1e-10):
    L, K, Df = cb.shape
    D, H, W = wmap.shape
    F = np.einsum("ldk,lkn->ldn", np.transpose(cb, (0, 2, 1)).astype(np.float64),
                  wmap.reshape(L, K, H * W).astype(np.float64)).reshape(L, Df, H, W)
    if normalize:
        F = F / (np.linalg.norm(F, axis=1, keepdims=True) + eps)
    return F


def test_validation_on_cpu():
    with pytest.raises(ValueError):
        quick.decode_language_features(torch.zeros(100, 4, 4), torch.zeros(3, 64, 512))
    with pytest.raises(ValueError):
        quick.decode_language_features(torch.zeros(4, 4), torch.zeros(3, 64, 512))
    with pytest.raises(RuntimeError, match="no CPU path"):
        quick.decode_language_features(torch.zeros(192, 4, 4), torch.zeros(3, 64, 512))


@pytest.mark.gpu
@pytest.mark.parametrize("H,W", [(37, 45), (64, 128), (1, 1)])
def test_decode_matches_float64(gpu, H, W):
    g = np.random.default_rng(H * 1000 + W)
    L, K, Df = 3, 64, 512
    # quick weights: sparse non-negative mixtures (top-k soft codes blended over depth)
    wmap = (g.random((L * K, H, W)) * (g.random((L * K, H, W)) < 0.15)).astype(np.float32)
    cb = g.standard_normal((L, K, Df)).astype(np.float32)
    got = quick.decode_language_features(torch.from_numpy(wmap).to(gpu), torch.from_numpy(cb).to(gpu))
    ref = ref_decode(wmap, cb)
    np.testing.assert_allclose(got.cpu().numpy(), ref, atol=DEC_ATOL, rtol=0)


@pytest.mark.gpu
def test_decode_subnormal_and_tiny_weights(gpu):
    """the per-pixel power-of-two scaling before the f16 split
    must stay finite when a pixel's largest weight is subnormal (or tiny):
    such a pixel decodes to ~0 as the reference's einsum / (norm + 1e-10)
    does, never to NaN/Inf; its neighbours are unaffected."""
    g = np.random.default_rng(11)
    L, K, Df, H, W = 3, 64, 512, 24, 40
    wmap = (g.random((L * K, H, W)) * (g.random((L * K, H, W)) < 0.2)).astype(np.float32)
    for (y, x), s in {(0, 0): 1e-40, (3, 5): 1e-44, (7, 9): 1e-30, (11, 20): 1e-20, (23, 39): 2e-38}.items():
        wmap[:, y, x] = (wmap[:, y, x].astype(np.float64) * s).astype(np.float32)
    cb = g.standard_normal((L, K, Df)).astype(np.float32)
    got = quick.decode_language_features(torch.from_numpy(wmap).to(gpu), torch.from_numpy(cb).to(gpu)).cpu().numpy()
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, ref_decode(wmap, cb), atol=DEC_ATOL, rtol=0)


@pytest.mark.gpu
def test_unnormalised_and_dense_map(gpu):
    g = np.random.default_rng(7)
    wmap = g.random((64, 40, 56)).astype(np.float32)
    cb = g.standard_normal((1, 64, 512)).astype(np.float32)
    got = quick.compute_final_feature_map(torch.from_numpy(wmap).to(gpu), torch.from_numpy(cb).to(gpu))
    ref = ref_decode(wmap, cb, normalize=False)[0]
    scale = np.abs(ref).max()
    np.testing.assert_allclose(got.cpu().numpy() / scale, ref / scale, atol=DEC_ATOL, rtol=0)


@pytest.mark.gpu
def test_render_then_decode_end_to_end(gpu, oracle_lib):
    """Quick render through the drop-in rasterizer (weights bit-exact vs the
    oracle) followed by the decode, vs the oracle's weight map decoded in float64."""
    from harness import make_case, run_gpu_forward, oracle_problem
    case = make_case(N=3000, W=96, H=80, seed=21, sh_degree=None, quick_k=4)
    ref_f = oracle_lib.forward(oracle_problem(case))
    got_f = run_gpu_forward(case, gpu)
    np.testing.assert_array_equal(got_f["lang"], ref_f["lang"])
    cb = np.random.default_rng(3).standard_normal((3, 64, 512)).astype(np.float32)
    feats = quick.decode_language_features(torch.from_numpy(got_f["lang"]).to(gpu), torch.from_numpy(cb).to(gpu))
    np.testing.assert_allclose(feats.cpu().numpy(), ref_decode(ref_f["lang"], cb), atol=DEC_ATOL, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(3, 64, 32), (1, 40, 48), (2, 96, 16)])
def test_final_feature_map_any_level_count(gpu, shape):
    """compute_final_feature_map accepts any number of levels / codes like the reference's
    codebooks.view(-1, Df).T @ W (scene/gaussian_model.py:545-550): 64-code blocks summed,
    R padded with zero codes to a multiple of 64."""
    g = np.random.default_rng(sum(shape))
    L, K, Df = shape
    wmap = g.random((L * K, 24, 40)).astype(np.float32)
    cb = g.standard_normal((L, K, Df)).astype(np.float32)
    got = quick.compute_final_feature_map(torch.from_numpy(wmap).to(gpu), torch.from_numpy(cb).to(gpu))
    ref = (cb.reshape(-1, Df).T.astype(np.float64) @ wmap.reshape(L * K, -1).astype(np.float64)).reshape(Df, 24, 40)
    scale = np.abs(ref).max()
    assert got.shape == (Df, 24, 40)
    np.testing.assert_allclose(got.cpu().numpy() / scale, ref / scale, atol=DEC_ATOL, rtol=0)


@pytest.mark.gpu
def test_plan_reuse_one_shot_and_invalidation(gpu):
    """lsr_quick_decode_prepare/_run (the per-codebook plan, cached by decode_plan)
    give the one-shot lsr_quick_decode's bits; an in-place codebook update (the
    tensor's version counter moves) prepares a new plan; a rank-deficient
    codebook (duplicated codes: a singular Gram matrix) still normalises."""
    import ctypes
    from langsplatv2_amd import _lib
    from langsplatv2_amd.rasterizer import _Alloc, _stream
    g = np.random.default_rng(3)
    L, K, Df, H, W = 3, 64, 512, 40, 52
    wmap = torch.from_numpy((g.random((L * K, H, W)) * (g.random((L * K, H, W)) < 0.2)).astype(np.float32)).to(gpu)
    cb = torch.from_numpy(g.standard_normal((L, K, Df)).astype(np.float32)).to(gpu)
    a = quick.decode_language_features(wmap, cb)
    b = quick.decode_language_features(wmap, cb)          # cached plan
    one = torch.empty_like(a)
    alloc = _Alloc(gpu)
    lib = _lib.load()
    _lib.check(lib.lsr_quick_decode(wmap.data_ptr(), cb.data_ptr(), L, K, Df, H, W, 1, ctypes.c_float(1e-10),
                                    one.data_ptr(), alloc.fn, None, _stream(gpu)), "lsr_quick_decode")
    assert torch.equal(a, b) and torch.equal(a, one)
    cb.mul_(-0.5)                                          # in place: version counter moves
    c = quick.decode_language_features(wmap, cb)
    np.testing.assert_allclose(c.cpu().numpy(), ref_decode(wmap.cpu().numpy(), cb.cpu().numpy()), atol=DEC_ATOL)
    cb2 = cb.clone()
    cb2[:, 32:] = cb2[:, :32]                              # rank 32 per level
    d = quick.decode_language_features(wmap, cb2)
    np.testing.assert_allclose(d.cpu().numpy(), ref_decode(wmap.cpu().numpy(), cb2.cpu().numpy()), atol=DEC_ATOL)


@pytest.mark.gpu
def test_plan_invalidated_by_fused_adam_step(gpu):
    """FusedAdam writes the codebooks through a raw pointer; it bumps their
    version counter, so the next decode prepares a new plan."""
    from langsplatv2_amd.optim import FusedAdam
    g = np.random.default_rng(11)
    L, K, Df, H, W = 3, 64, 512, 24, 32
    wmap = torch.from_numpy((g.random((L * K, H, W)) * (g.random((L * K, H, W)) < 0.2)).astype(np.float32)).to(gpu)
    cb = torch.from_numpy(g.standard_normal((L, K, Df)).astype(np.float32)).to(gpu).requires_grad_(True)
    quick.decode_language_features(wmap, cb.detach())
    v0 = cb._version
    opt = FusedAdam([cb], lr=0.05)
    cb.grad = torch.randn(cb.shape, generator=torch.Generator().manual_seed(1)).to(gpu)
    opt.step()
    assert cb._version > v0
    got = quick.decode_language_features(wmap, cb.detach())
    np.testing.assert_allclose(got.cpu().numpy(), ref_decode(wmap.cpu().numpy(), cb.detach().cpu().numpy()),
                               atol=DEC_ATOL)
