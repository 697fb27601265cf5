"""The feature-phase loss under train.py's other flags (train.py:151-167):
--normalize, --l1_loss, both losses summed, and layer_idx > 0
(compute_layer_feature_map, scene/gaussian_model.py:533-543, earlier levels
detached).  Reference: a float64 restatement of those lines in torch on the
CPU (test infrastructure), differentiated by autograd.  Tolerances: the loss
within 2e-6 absolute, gradients within 1e-5 x max|ref| + 1e-8 (fp32 GEMMs over
512-wide features, the fused kernel's code-space factorisation)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from langsplatv2_amd.lang_loss import language_feature_loss

LOSS_ATOL = 2e-6
GRAD_RTOL = 1e-5


def ref_loss(wm, cb, seg, feat, layer_idx, normalize, cos, l1):
    """train.py:155-167 in float64 (scene/gaussian_model.py:533-543, scene/cameras.py:77-94,
    utils/loss_utils.py:18-25)."""
    D, H, W = wm.shape
    L, K, Df = cb.shape
    w = wm.reshape(D, -1)
    f = None
    for i in range(layer_idx + 1):
        fi = (cb[i].T @ w[i * K:(i + 1) * K]).view(Df, H, W)
        f = fi if f is None else fi + f.detach()
    if normalize:
        f = f / (f.norm(dim=0, keepdim=True) + 1e-10)
    sg = seg.long()
    mask = (sg != -1).unsqueeze(0)
    gt = feat[sg].permute(2, 0, 1)
    loss = torch.zeros((), dtype=torch.float64)
    if cos:
        loss = loss + 1 - F.cosine_similarity(f * mask, gt * mask, dim=0).mean()
    if l1:
        loss = loss + (f * mask - gt * mask).abs().mean()
    return loss


def _problem(L=1, H=37, W=53, S=23, seed=0):
    g = torch.Generator().manual_seed(seed)
    wm = torch.rand(L * 64, H, W, generator=g) * (torch.rand(L * 64, H, W, generator=g) < 0.2)
    cb = torch.randn(L, 64, 512, generator=g)
    feat = torch.randn(S, 512, generator=g)
    seg = torch.randint(-1, S, (H, W), generator=g, dtype=torch.int32)
    return wm, cb, seg, feat


def test_variant_validation_on_cpu():
    wm, cb, seg, feat = _problem()
    with pytest.raises(ValueError, match="layer_idx"):
        language_feature_loss(wm, cb, seg, feat, layer_idx=1)
    with pytest.raises(ValueError, match="at least one"):
        language_feature_loss(wm, cb, seg, feat, cos=False, l1=False)
    with pytest.raises(RuntimeError, match="no CPU path"):
        language_feature_loss(wm, cb, seg, feat, l1=True)


@pytest.mark.gpu
@pytest.mark.parametrize("L,layer_idx,normalize,cos,l1", [
    (1, 0, True, True, False),    # --normalize --cos_loss: the fused kernel
    (1, 0, False, False, True),   # --l1_loss
    (1, 0, True, True, True),     # --normalize --cos_loss --l1_loss
    (2, 1, False, True, False),   # layer_idx 1 (two codebook levels)
    (3, 2, True, True, True),
])
def test_loss_variants_match_reference(gpu, L, layer_idx, normalize, cos, l1):
    wm, cb, seg, feat = _problem(L=L, seed=L * 10 + layer_idx)
    w64 = wm.double().requires_grad_(True)
    c64 = cb.double().requires_grad_(True)
    ref = ref_loss(w64, c64, seg, feat.double(), layer_idx, normalize, cos, l1)
    ref.backward()
    wg = wm.to(gpu).requires_grad_(True)
    cg = cb.to(gpu).requires_grad_(True)
    got = language_feature_loss(wg, cg, seg.to(gpu), feat.to(gpu), layer_idx=layer_idx, normalize=normalize,
                                cos=cos, l1=l1)
    got.backward()
    assert abs(float(got.detach()) - float(ref)) <= LOSS_ATOL, (float(got.detach()), float(ref))
    for name, a, b in (("weight_map", wg.grad, w64.grad), ("codebooks", cg.grad, c64.grad)):
        a = a.double().cpu().numpy()
        b = b.numpy()
        err = np.abs(a - b).max()
        assert err <= GRAD_RTOL * max(np.abs(b).max(), 1e-3) + 1e-8, (name, err, np.abs(b).max())
    # the earlier levels take no gradient (compute_layer_feature_map detaches them)
    if layer_idx > 0:
        assert float(cg.grad[:layer_idx].abs().max()) == 0.0
        assert float(wg.grad[:layer_idx * 64].abs().max()) == 0.0


@pytest.mark.gpu
def test_trainer_step_with_l1_and_normalize(gpu):
    """LanguageTrainer (one rank) with --normalize --cos_loss --l1_loss takes the
    step accumulate_language_views takes with those flags: the same loss, and
    gradients equal up to the rasterizer backward's float-atomic summation
    order (the parameters after Adam are not compared: with eps 1e-15 it turns
    the rounding noise on zero-signal logits into +-lr steps, see
    test_0_train_dp_lang.py)."""
    from langsplatv2_amd.train_loop import LanguageTrainer, accumulate_language_views
    from test_0_train_dp_lang import _scene
    flags = dict(normalize=True, cos=True, l1=True)
    cams, segs, feats, ls_a = _scene(gpu)
    _, _, _, ls_b = _scene(gpu)
    tr = LanguageTrainer(ls_a, torch.zeros(3, device=gpu), normalize=True, cos_loss=True, l1_loss=True)
    la = tr.step(cams[0], segs[0], feats[0])
    ga = [g.detach().clone() for g in tr.last_grads]
    gb = []
    lb = accumulate_language_views(ls_b, ls_b.optimizer(), [cams[0]], [segs[0]], [feats[0]],
                                   torch.zeros(3, device=gpu), grads_out=gb, **flags)
    assert np.isfinite(la) and la == lb[0]
    for a, b in zip(ga, gb):
        assert float(b.abs().max()) > 0.0
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()) + 1e-12
