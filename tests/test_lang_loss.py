"""Fused language-feature cosine loss (csrc/lang_loss.hip).

CPU: the oracle restatement (oracle.lang_cos_loss) against vectors produced by
the reference's own cos_loss (tests/golden/make_lang_loss_golden.py).
GPU: langsplatv2_amd.lang_loss.language_cos_loss (forward + autograd
backward through the C ABI) against the golden vectors and the oracle.
Tolerances (fp32 kernel vs float64 references): loss 2e-7 absolute;
dL/dweight_map per pixel 2e-6 of that pixel's largest |gradient| (the
|f| = 0 pixel's gradient is ~1e6, the rest ~1e-3); dL/dcodebooks 2e-6 of the
largest |entry|.  Measured (tools/loss_err.py -> profiles/r03_loss_err.json,
these cases + 270x480): loss <= 2.8e-8, dL/dW <= 6.3e-7, dL/dcodebooks
<= 6.0e-7; the reference's own fp32 formulation (cos_loss on the materialised
(512, H, W) maps, torch on the same GPU) is off the float64 truth by up to
2.3e-6 (dL/dW) and 6.2e-6 (dL/dcodebooks) on the same cases.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_lang_loss.npz")
LOSS_ATOL = 2e-7
GRAD_RTOL = 2e-6


def _gold(name):
    z = np.load(GOLD)
    return {k[len(name) + 1:]: z[k] for k in z.files if k.startswith(name + "_")}


def assert_grad_w(got, ref):
    K = ref.shape[0]
    g = got.reshape(K, -1).astype(np.float64)
    r = ref.reshape(K, -1)
    scale = np.maximum(np.abs(r).max(0), 1e-12)
    err = (np.abs(g - r).max(0) / scale).max()
    assert err <= GRAD_RTOL, f"dL/dweight_map: worst per-pixel relative error {err:.3g}"


def assert_grad_cb(got, ref):
    err = np.abs(got.astype(np.float64) - ref).max() / max(np.abs(ref).max(), 1e-30)
    assert err <= GRAD_RTOL, f"dL/dcodebooks: relative error {err:.3g}"


@pytest.mark.parametrize("name", ["a", "b"])
def test_oracle_matches_reference_cos_loss(name):
    z = _gold(name)
    loss, dW, dcb = O.lang_cos_loss(z["weight_map"], z["codebooks"][0], z["seg"], z["features"])
    assert abs(loss - float(z["loss"])) < 1e-12
    np.testing.assert_allclose(dW, z["grad_weight_map"], rtol=1e-9, atol=1e-9 * np.abs(z["grad_weight_map"]).max())
    np.testing.assert_allclose(dcb, z["grad_codebooks"][0], rtol=1e-9, atol=1e-12)


def _random_case(K, Df, H, W, S, seed):
    rng = np.random.default_rng(seed)
    wm = rng.random((K, H, W)) ** 3
    wm /= wm.sum(0, keepdims=True) + 1e-3
    cb = rng.standard_normal((K, Df))
    feat = rng.standard_normal((S, Df))
    # spatially coherent segments (SAM-like regions), some masked
    yy, xx = np.mgrid[0:H, 0:W]
    seg = ((yy // 7) * 5 + (xx // 11)) % (S + 1) - 1
    return wm.astype(np.float32), cb.astype(np.float32), seg.astype(np.int32), feat.astype(np.float32)


def _gpu_loss(wm, cb, seg, feat, scale=1.0):
    from langsplatv2_amd.lang_loss import language_cos_loss
    dev = torch.device("cuda:0")
    w = torch.from_numpy(wm).to(dev).requires_grad_(True)
    c = torch.from_numpy(cb).to(dev).requires_grad_(True)
    loss = language_cos_loss(w, c, torch.from_numpy(seg).to(dev), torch.from_numpy(feat).to(dev))
    (loss * scale).backward()
    return loss.item(), w.grad.cpu().numpy(), c.grad.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["a", "b"])
def test_gpu_matches_reference_golden(name):
    z = _gold(name)
    loss, gw, gcb = _gpu_loss(z["weight_map"], z["codebooks"], z["seg"], z["features"])
    assert abs(loss - float(z["loss"])) <= LOSS_ATOL
    assert_grad_w(gw, z["grad_weight_map"])
    assert_grad_cb(gcb[0], z["grad_codebooks"][0])


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,S,seed", [(67, 93, 40, 0), (128, 128, 5, 1), (4, 16, 1, 2), (33, 250, 300, 3)])
def test_gpu_matches_oracle(H, W, S, seed):
    wm, cb, seg, feat = _random_case(64, 512, H, W, S, seed)
    ref_loss, ref_w, ref_cb = O.lang_cos_loss(wm, cb, seg, feat)
    loss, gw, gcb = _gpu_loss(wm, cb, seg, feat)
    assert abs(loss - ref_loss) <= LOSS_ATOL
    assert_grad_w(gw, ref_w)
    assert_grad_cb(gcb, ref_cb)


@pytest.mark.gpu
def test_gpu_upstream_scale_and_all_masked():
    wm, cb, seg, feat = _random_case(64, 256, 20, 40, 6, 4)
    ref_loss, ref_w, ref_cb = O.lang_cos_loss(wm, cb, seg, feat)
    loss, gw, gcb = _gpu_loss(wm, cb, seg, feat, scale=-2.5)
    assert_grad_w(gw, -2.5 * ref_w)
    assert_grad_cb(gcb, -2.5 * ref_cb)
    # every pixel masked: loss 1, zero gradients
    seg[:] = -1
    loss, gw, gcb = _gpu_loss(wm, cb, seg, feat)
    assert loss == 1.0 and not gw.any() and not gcb.any()


@pytest.mark.gpu
def test_gpu_rejects_bad_shapes():
    from langsplatv2_amd.lang_loss import language_cos_loss
    dev = torch.device("cuda:0")
    with pytest.raises(ValueError):
        language_cos_loss(torch.zeros(32, 4, 4, device=dev), torch.zeros(32, 512, device=dev),
                          torch.zeros(4, 4, dtype=torch.int32, device=dev), torch.zeros(2, 512, device=dev))
    with pytest.raises(ValueError):
        language_cos_loss(torch.zeros(64, 4, 4, device=dev), torch.zeros(64, 512, device=dev),
                          torch.zeros(4, 5, dtype=torch.int32, device=dev), torch.zeros(2, 512, device=dev))
