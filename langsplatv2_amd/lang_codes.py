"""Language-coefficient producers on the rasterizer's input edge.

Restatements (torch, device-agnostic) of utils/vq_utils.py:
  softmax_to_topk_soft_code  :9-24  -> dense (N, K) with k non-zeros per row
  get_weights_and_indices    :26-40 -> packed (N, k) weights, (N, k) fp32 indices
                                       in ascending channel order (mask order)
and of GaussianModel.get_render_weights (scene/gaussian_model.py:510-518).
Golden vectors from the reference's own functions pin them
(tests/golden/ref_utils.npz, tests/test_ref_golden.py).
"""
from __future__ import annotations

import torch


def softmax_to_topk_soft_code(logits: torch.Tensor, k: int) -> torch.Tensor:
    y = logits.softmax(dim=1)
    _, idx = torch.topk(y, k, dim=1)
    mask = torch.zeros_like(y, dtype=torch.bool).scatter_(1, idx, True)
    y = torch.where(mask, y, torch.zeros_like(y))
    return y / (y.sum(dim=1, keepdim=True) + 1e-10)


def get_weights_and_indices(logits: torch.Tensor, k: int):
    code = softmax_to_topk_soft_code(logits, k)
    nz = code != 0
    w = code[nz].view(code.shape[0], k)
    i = torch.arange(code.shape[1], device=code.device).expand_as(code)[nz].view(code.shape[0], k)
    return w.float(), i.float()


def get_render_weights(logits: torch.Tensor, layer_num: int, codebook_size: int, k: int) -> torch.Tensor:
    """Per-level top-k soft codes concatenated -> (N, layer_num*codebook_size)."""
    parts = [softmax_to_topk_soft_code(logits[:, i * codebook_size:(i + 1) * codebook_size], k)
             for i in range(layer_num)]
    return torch.cat(parts, dim=-1).float()
