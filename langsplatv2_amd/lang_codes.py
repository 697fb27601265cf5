"""Top-k soft codes on the rasterizer's language input edge, fused on the GPU.

One HIP kernel (csrc/lang_codes.hip, C ABI lsr_topk_code_forward/backward)
replaces the reference's chains of PyTorch ops:
  softmax_to_topk_soft_code  utils/vq_utils.py:9-24   -> dense (N, K), k non-zeros per row
  get_weights_and_indices    utils/vq_utils.py:26-40  -> packed (N, k) weights + fp32
                                                         indices in ascending channel order
  get_render_weights         scene/gaussian_model.py:510-518 (per-level concatenation)
  quick_inputs               eval_lerf.py:340-348, backend_renderer.py:121-128
                             (levels' packed codes, indices offset by 64*level)
The dense codes are differentiable w.r.t. the logits (the backward is the
same autograd chain torch applies, computed by a second fused kernel).
There is no CPU path; ties in the top-k go to the lower channel.
"""
from __future__ import annotations

import torch

from . import _lib
from .rasterizer import _stream


def _check_logits(logits: torch.Tensor, levels: int, what: str) -> tuple[torch.Tensor, int, int]:
    if logits.dim() != 2:
        raise ValueError(f"{what}: logits must be (N, levels*K), got {tuple(logits.shape)}")
    if not logits.is_cuda:
        raise RuntimeError(f"{what}: logits must be a ROCm device tensor (there is no CPU path)")
    N, LK = logits.shape
    if levels < 1 or LK % levels:
        raise ValueError(f"{what}: {LK} channels do not split into {levels} levels")
    return logits.contiguous().float(), N, LK // levels


class _TopkSoftCode(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, k, levels):
        x, N, K = _check_logits(logits, levels, "softmax_to_topk_soft_code")
        out = torch.empty_like(x)
        lib = _lib.load()
        _lib.check(lib.lsr_topk_code_forward(x.data_ptr(), N, levels, K, int(k), out.data_ptr(), None, None,
                                             _lib.LSR_INDEX_F32, 0, _stream(x.device)), "lsr_topk_code_forward")
        ctx.save_for_backward(x)
        ctx.k, ctx.levels = int(k), levels
        return out

    @staticmethod
    def backward(ctx, grad):
        (x,) = ctx.saved_tensors
        N, LK = x.shape
        g = grad.contiguous().float()
        dx = torch.empty_like(x)
        lib = _lib.load()
        _lib.check(lib.lsr_topk_code_backward(x.data_ptr(), g.data_ptr(), N, ctx.levels, LK // ctx.levels, ctx.k,
                                              dx.data_ptr(), _stream(x.device)), "lsr_topk_code_backward")
        return dx, None, None


def softmax_to_topk_soft_code(logits: torch.Tensor, k: int) -> torch.Tensor:
    """utils/vq_utils.py:9-24 -> (N, K) fp32, differentiable w.r.t. logits."""
    return _TopkSoftCode.apply(logits, k, 1)


def get_render_weights(logits: torch.Tensor, layer_num: int, codebook_size: int, k: int) -> torch.Tensor:
    """scene/gaussian_model.py:510-518: per-level top-k soft codes of
    logits (N, layer_num*codebook_size), concatenated -> (N, layer_num*codebook_size)."""
    if logits.shape[-1] != layer_num * codebook_size:
        raise ValueError(f"get_render_weights: logits have {logits.shape[-1]} channels, "
                         f"expected {layer_num}*{codebook_size}")
    return _TopkSoftCode.apply(logits, k, layer_num)


def quick_inputs(logits: torch.Tensor, k: int, levels: int = 1, level_offset: bool = True,
                 index_dtype: torch.dtype = torch.float32):
    """Packed sparse codes of every level: (weights (N, levels*k) fp32, indices
    (N, levels*k) of index_dtype), indices + K*level when level_offset —
    the language_feature_weights_quick / language_feature_indices pair of
    eval_lerf.py:340-348.  Not differentiable (every quick caller is no_grad;
    `sparse_codes` is the differentiable form)."""
    with torch.no_grad():
        return _quick_inputs_impl(logits, k, levels, level_offset, index_dtype)


def _quick_inputs_impl(logits, k, levels, level_offset, index_dtype):
    x, N, K = _check_logits(logits, levels, "quick_inputs")
    codes = {torch.float32: _lib.LSR_INDEX_F32, torch.int32: _lib.LSR_INDEX_I32, torch.int64: _lib.LSR_INDEX_I64}
    if index_dtype not in codes:
        raise ValueError(f"quick_inputs: index dtype {index_dtype} unsupported (float32/int32/int64)")
    w = torch.empty((N, levels * k), dtype=torch.float32, device=x.device)
    idx = torch.empty((N, levels * k), dtype=index_dtype, device=x.device)
    lib = _lib.load()
    _lib.check(lib.lsr_topk_code_forward(x.data_ptr(), N, levels, K, int(k), None, w.data_ptr(), idx.data_ptr(),
                                         codes[index_dtype], int(bool(level_offset)), _stream(x.device)),
               "lsr_topk_code_forward")
    return w, idx


class _TopkSparse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, k, levels, level_offset, index_dtype):
        w, idx = _quick_inputs_impl(logits, k, levels, level_offset, index_dtype)
        ctx.save_for_backward(logits.contiguous().float())
        ctx.k, ctx.levels = int(k), levels
        ctx.mark_non_differentiable(idx)
        return w, idx

    @staticmethod
    def backward(ctx, gw, _gidx):
        (x,) = ctx.saved_tensors
        N, LK = x.shape
        dx = torch.empty_like(x)
        if gw is None:
            return dx.zero_(), None, None, None, None
        g = gw.contiguous().float()
        lib = _lib.load()
        _lib.check(lib.lsr_topk_code_backward_sparse(x.data_ptr(), g.data_ptr(), N, ctx.levels, LK // ctx.levels,
                                                     ctx.k, dx.data_ptr(), _stream(x.device)),
                   "lsr_topk_code_backward_sparse")
        return dx, None, None, None, None


def sparse_codes(logits: torch.Tensor, k: int, levels: int = 1, level_offset: bool = True,
                 index_dtype: torch.dtype = torch.int32):
    """The packed top-k codes as a DIFFERENTIABLE rasterizer input:
    (weights (N, levels*k) fp32 with grad w.r.t. logits, indices (N, levels*k)), the
    language_feature_weights_quick / language_feature_indices pair rendered with
    quick_render=True and language_feature_dim = levels*K.  Feature-mode training
    then never forms the dense (N, K) codes (get_render_weights, scene/gaussian_model.py:
    510-518): the rasterizer returns dL/dweights (N, levels*k) and the producer's
    sparse backward turns it into dL/dlogits.  Mathematically the same gradient as
    the dense path: dL/dw[j][m] = dL/dcode[j][idx[j][m]] and the unselected codes
    are constant zeros."""
    return _TopkSparse.apply(logits, k, levels, level_offset, index_dtype)


def get_weights_and_indices(logits: torch.Tensor, k: int):
    """utils/vq_utils.py:26-40: (weights (N, k) fp32, indices (N, k) fp32) in
    ascending channel order."""
    with torch.no_grad():
        return quick_inputs(logits, k, 1, level_offset=False)
