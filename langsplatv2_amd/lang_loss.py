"""Language-feature loss of the feature-mode training step, fused on the GPU.

The reference's per-iteration loss after render() (train.py:151-164,
vq_layer_num = 1 as in train.sh, so layer_idx = 0):

    gt, mask = viewpoint_cam.get_language_feature(lf_path, feature_level)   scene/cameras.py:59-96
        # gt[:, p] = feature_map[seg[p]] from <image>_f.npy / <image>_s.npy; mask = seg != -1
    f = gaussians.compute_layer_feature_map(weight_map, 0)                   scene/gaussian_model.py:533-543
        # f = codebooks[0].T @ weight_map.view(K, -1)      (512, H, W)
    loss = cos_loss(f * mask, gt * mask)                                     utils/loss_utils.py:24-25

`language_cos_loss` computes the same loss and its gradients w.r.t. the
weight map and the codebooks with one HIP pass per direction
(csrc/lang_loss.hip, C ABI lsr_lang_loss_forward/backward): the (512, H, W)
feature, ground-truth and product tensors the reference materialises are
never formed (every quantity factors through the 64-dim code space), and the
ground truth is read as per-pixel segment ids into a per-view (S, 512)
feature table instead of a gathered (512, H, W) map.  There is no CPU path.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .rasterizer import _Alloc, _stream


def language_gt_index(seg_maps, feature_level: int, device=None) -> torch.Tensor:
    """The segment-id form of get_language_feature's ground truth
    (scene/cameras.py:77-94): row `feature_level` of the (levels, H, W)
    `<image>_s.npy` map as an int32 (H, W) device tensor; -1 = masked.  The
    matching feature table is `<image>_f.npy` as an (S, 512) fp32 tensor.
    (The reference's nearest-neighbour resize for mismatched sizes needs cv2
    and is not reproduced.)"""
    if feature_level not in (0, 1, 2, 3):
        raise ValueError(f"feature_level={feature_level}")
    s = seg_maps if isinstance(seg_maps, torch.Tensor) else torch.from_numpy(np.asarray(seg_maps))
    return s[feature_level].to(device=device, dtype=torch.int32).contiguous()


def _args(weight_map, codebooks, seg, features):
    if weight_map.dim() != 3:
        raise ValueError("language_cos_loss: weight_map must be (K, H, W)")
    cb = codebooks[0] if codebooks.dim() == 3 else codebooks
    if cb.dim() != 2:
        raise ValueError("language_cos_loss: codebooks must be (layers, K, Df) or (K, Df)")
    K, H, W = weight_map.shape
    if cb.shape[0] != K:
        raise ValueError(f"language_cos_loss: weight_map has {K} channels, the codebook {cb.shape[0]} codes")
    if K != 64 or cb.shape[1] % 16:
        raise ValueError("language_cos_loss: K must be 64 (codebook_size of train.sh) and Df a multiple of 16")
    if tuple(seg.shape) != (H, W):
        raise ValueError(f"language_cos_loss: seg must be (H, W) = {(H, W)}, got {tuple(seg.shape)}")
    if features.dim() != 2 or features.shape[1] != cb.shape[1]:
        raise ValueError("language_cos_loss: features must be (S, Df) with the codebook's Df")
    for t, n in ((weight_map, "weight_map"), (cb, "codebooks"), (seg, "seg"), (features, "features")):
        if not t.is_cuda:
            raise RuntimeError(f"language_cos_loss: {n} must be a ROCm device tensor (there is no CPU path)")
    return (weight_map.detach().contiguous().float(), cb.detach().contiguous().float(),
            seg.detach().to(torch.int32).contiguous(), features.detach().contiguous().float(), K, H, W)


class _LanguageCosLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight_map, codebooks, seg, features):
        wm, cb, sg, ft, K, H, W = _args(weight_map, codebooks, seg, features)
        loss = torch.empty((1,), dtype=torch.float32, device=wm.device)
        stats = torch.empty((2, H, W), dtype=torch.float32, device=wm.device)   # |f_p|, f_p.gt_p
        alloc = _Alloc(wm.device)
        _lib.check(_lib.load().lsr_lang_loss_forward(wm.data_ptr(), cb.data_ptr(), K, cb.shape[1], H, W,
                                                     sg.data_ptr(), ft.data_ptr(), ft.shape[0], loss.data_ptr(),
                                                     stats.data_ptr(), alloc.fn, None, _stream(wm.device)),
                   "lsr_lang_loss_forward")
        ctx.save_for_backward(wm, cb, sg, ft, stats)
        ctx.cb_shape = tuple(codebooks.shape)
        return loss[0]

    @staticmethod
    def backward(ctx, grad):
        wm, cb, sg, ft, stats = ctx.saved_tensors
        K, H, W = wm.shape
        g = grad.detach().reshape(1).contiguous().float()
        gw = torch.empty_like(wm)
        gcb = torch.empty_like(cb)
        alloc = _Alloc(wm.device)
        _lib.check(_lib.load().lsr_lang_loss_backward(wm.data_ptr(), cb.data_ptr(), K, cb.shape[1], H, W,
                                                      sg.data_ptr(), ft.data_ptr(), ft.shape[0], stats.data_ptr(),
                                                      g.data_ptr(), gw.data_ptr(), gcb.data_ptr(), alloc.fn, None,
                                                      _stream(wm.device)), "lsr_lang_loss_backward")
        if len(ctx.cb_shape) == 3:   # layers > 0 take no part at layer_idx 0
            full = torch.zeros(ctx.cb_shape, dtype=gcb.dtype, device=gcb.device)
            full[0] = gcb
            gcb = full
        return (gw if ctx.needs_input_grad[0] else None, gcb if ctx.needs_input_grad[1] else None, None, None)


def language_cos_loss(weight_map: torch.Tensor, codebooks: torch.Tensor, seg: torch.Tensor,
                      features: torch.Tensor) -> torch.Tensor:
    """1 - mean_p cos(f_p * m_p, gt_p * m_p) with f = codebooks[0].T @ weight_map,
    gt_p = features[seg_p], m_p = (0 <= seg_p < S); weight_map (64, H, W),
    codebooks (layers, 64, Df) or (64, Df), seg (H, W) int, features (S, Df).
    Differentiable w.r.t. weight_map and codebooks."""
    return _LanguageCosLoss.apply(weight_map, codebooks, seg, features)


def language_feature_loss(weight_map: torch.Tensor, codebooks: torch.Tensor, seg: torch.Tensor,
                          features: torch.Tensor, layer_idx: int = 0, normalize: bool = False, cos: bool = True,
                          l1: bool = False) -> torch.Tensor:
    """The feature-phase loss of train.py:151-167 under each of its flags:

        f = gaussians.compute_layer_feature_map(weight_map, layer_idx)     scene/gaussian_model.py:533-543
            # sum over levels i <= layer_idx of codebooks[i].T @ W[i K:(i+1) K], earlier levels detached
        if --normalize: f = f / (f.norm(dim=0, keepdim=True) + 1e-10)
        loss = [--cos_loss] cos_loss(f * mask, gt * mask) + [--l1_loss] l1_loss(f * mask, gt * mask)

    weight_map (L*K, H, W) (the rasterizer's dense language map), codebooks
    (L, K, Df), seg (H, W) int segment ids (-1 = masked), features (S, Df).

    The configuration train.sh trains with (layer 0, cosine loss; vq_layer_num
    1) runs the fused kernel (`language_cos_loss`); so does --normalize with the
    cosine loss alone, because the cosine of a per-pixel rescaled feature is
    the cosine of the feature (the only difference is the 1e-10 added to the
    norm: relative 1e-10 / |f_p|, far below fp32 resolution for any pixel with
    |f_p| > 1e-3; tests/test_lang_loss_variants.py).  The other flags (--l1_loss,
    the elementwise L1 over Df x H x W, and layer_idx > 0) are the reference's
    own tensor formulation on the device (torch ops over the Df-wide map)."""
    if codebooks.dim() != 3:
        raise ValueError("language_feature_loss: codebooks must be (layers, K, Df)")
    L, K, Df = codebooks.shape
    D, H, W = weight_map.shape
    if D < (layer_idx + 1) * K or not (0 <= layer_idx < L):
        raise ValueError(f"language_feature_loss: layer_idx {layer_idx} needs levels 0..{layer_idx} of the "
                         f"{L} codebooks and {(layer_idx + 1) * K} weight-map channels (got {D})")
    if not (cos or l1):
        raise ValueError("language_feature_loss: at least one of cos / l1 (train.py:161-167 sums them)")
    if layer_idx == 0 and cos and not l1:
        return language_cos_loss(weight_map[:K], codebooks, seg, features)
    for t, n in ((weight_map, "weight_map"), (codebooks, "codebooks"), (seg, "seg"), (features, "features")):
        if not t.is_cuda:
            raise RuntimeError(f"language_feature_loss: {n} must be a ROCm device tensor (there is no CPU path)")
    wm = weight_map.reshape(D, -1)
    f = None
    for i in range(layer_idx + 1):   # compute_layer_feature_map
        fi = (codebooks[i].T @ wm[i * K:(i + 1) * K]).view(Df, H, W)
        f = fi if f is None else fi + f.detach()
    if normalize:
        f = f / (f.norm(dim=0, keepdim=True) + 1e-10)
    S = features.shape[0]
    sg = seg.long()
    mask = (sg != -1).unsqueeze(0)                                   # scene/cameras.py:80
    gt = features[sg].permute(2, 0, 1)                               # features[-1] where masked, as the reference
    fm, gm = f * mask, gt * mask
    loss = torch.zeros((), dtype=f.dtype, device=f.device)
    if cos:
        loss = loss + (1 - torch.nn.functional.cosine_similarity(fm, gm, dim=0).mean())   # utils/loss_utils.py:24-25
    if l1:
        loss = loss + (fm - gm).abs().mean()                                          # utils/loss_utils.py:18-19
    return loss
