"""Codebook decode of rendered language weight maps on the MI355X matrix cores.

The reference decodes the rasterizer's language weight map in PyTorch after
render() (eval_lerf.py:210-220, backend_renderer.py:16-36):

    W = weight_map.view(L, K, H * W)
    F = torch.einsum('ldk,lkn->ldn', codebooks.permute(0, 2, 1), W).view(L, Df, H, W)
    F = F / (F.norm(dim=1, keepdim=True) + 1e-10)

and, for the dense training/eval map, compute_final_feature_map
(scene/gaussian_model.py:545-550): codebooks.view(-1, Df).T @ W.

`decode_language_features` does both in one HIP kernel per frame
(csrc/quick.hip: split-f16 MFMA with f32 accumulation, per-pixel norms from
the Cholesky factor of the codebook Gram matrix, each output written once);
the codebook-only preparation is cached per codebook tensor (`decode_plan`).
There is no CPU path.
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from . import _lib
from .rasterizer import _stream


def decode_language_features(weight_map: torch.Tensor, codebooks: torch.Tensor, normalize: bool = True,
                             eps: float = 1e-10, out: torch.Tensor | None = None) -> torch.Tensor:
    """weight_map (L*K, H, W) fp32 CUDA, codebooks (L, K, Df) fp32 CUDA ->
    features (L, Df, H, W); L2-normalised over Df per pixel when `normalize`.
    A pixel-major weight map (strides (1, L*K*W, L*K): the rasterizer's
    language_feature_layout="hwc" output) is read as it is (LSR_LAYOUT_HWC).
    `out`: an optional contiguous fp32 (L, Df, H, W) tensor to write into."""
    if weight_map.dim() != 3 or codebooks.dim() != 3:
        raise ValueError("decode_language_features: weight_map must be (L*K, H, W) and codebooks (L, K, Df)")
    L, K, Df = codebooks.shape
    D, H, W = weight_map.shape
    if D != L * K:
        raise ValueError(f"decode_language_features: weight_map has {D} channels, codebooks need L*K = {L * K}")
    if not (weight_map.is_cuda and codebooks.is_cuda):
        raise RuntimeError("decode_language_features: tensors must be on the ROCm device (there is no CPU path)")
    if K != 64 or Df % 16 != 0:
        raise ValueError("decode_language_features: K must be 64 and Df a multiple of 16")
    hwc = (weight_map.dtype == torch.float32 and weight_map.stride() == (1, D * W, D) and Df <= 512
           and weight_map.data_ptr() % 16 == 0 and H * W > 1)
    wm = weight_map if hwc else weight_map.contiguous().float()
    cb = codebooks.contiguous().float()
    if out is None:
        out = torch.empty((L, Df, H, W), dtype=torch.float32, device=weight_map.device)
    elif (tuple(out.shape) != (L, Df, H, W) or out.dtype != torch.float32 or not out.is_contiguous()
          or out.device != weight_map.device):
        raise ValueError(f"decode_language_features: out must be a contiguous float32 ({L}, {Df}, {H}, {W}) tensor")
    lib = _lib.load()
    plan = decode_plan(cb, normalize)
    rc = lib.lsr_quick_decode_run(wm.data_ptr(), _lib.LSR_LAYOUT_HWC if hwc else _lib.LSR_LAYOUT_CHW,
                                  plan.data_ptr(), L, K, Df, H, W, int(bool(normalize)), float(eps),
                                  out.data_ptr(), _stream(weight_map.device))
    _lib.check(rc, "lsr_quick_decode_run")
    return out


_PLANS: "OrderedDict[tuple, tuple]" = OrderedDict()
_PLAN_CACHE_SIZE = 4


def decode_plan(codebooks: torch.Tensor, normalize: bool = True) -> torch.Tensor:
    """The codebook-only part of the decode (MFMA fragments, Cholesky factor of
    the Gram matrix for the norm), prepared once per codebook tensor and reused
    for every frame (lsr_quick_decode_prepare).  Cached by the tensor's storage,
    shape and version counter, so an in-place update of the codebooks (an
    optimizer step) prepares a new plan."""
    cb = codebooks.contiguous().float()
    L, K, Df = cb.shape
    key = (cb.data_ptr(), cb.device, tuple(cb.shape), cb._version, bool(normalize))
    hit = _PLANS.get(key)
    if hit is not None:
        _PLANS.move_to_end(key)
        return hit[1]
    lib = _lib.load()
    nbytes = int(lib.lsr_quick_decode_plan_bytes(L, K, Df, int(bool(normalize))))
    if nbytes == 0:
        raise ValueError("decode_plan: unsupported codebook shape")
    plan = torch.empty(nbytes, dtype=torch.uint8, device=cb.device)
    _lib.check(lib.lsr_quick_decode_prepare(cb.data_ptr(), L, K, Df, int(bool(normalize)), plan.data_ptr(),
                                            _stream(cb.device)), "lsr_quick_decode_prepare")
    _PLANS[key] = (cb, plan)   # the reference keeps the storage (and its data_ptr) alive
    while len(_PLANS) > _PLAN_CACHE_SIZE:
        _PLANS.popitem(last=False)
    return plan


class QuickFeatureStream:
    """Render + decode over a stream of views, frame i's decode overlapping
    frame i+1's render.  The reference evaluates view after view, each as
    render -> einsum -> normalise (eval_lerf.py:210-220, :320-350;
    backend_renderer.py:16-36).  The quick render is latency-bound (2 waves per
    SIMD, its HBM traffic ~1 GB per 1-Mpix frame) and the decode HBM-bound
    (7.08 GB per frame), so running them back to back leaves each one's
    resources idle while the other runs.  Here the decode goes to a second HIP
    stream and the caller's stream goes on to the next render; the features
    of frame i come back from the push of frame i + 1 (or from `flush`), made
    safe to use on the caller's stream.

        fs = QuickFeatureStream(codebooks)
        for view in views:
            prev = fs.push(lambda: render(view, ...)["language_feature_weight_map"])
            if prev is not None:
                use(prev)                   # (L, Df, H, W), the previous view's
        use(fs.flush())

    Each frame's values equal decode_language_features(weight map) exactly (the
    same kernels; only the issue order differs)."""

    def __init__(self, codebooks: torch.Tensor, normalize: bool = True, eps: float = 1e-10):
        self.codebooks, self.normalize, self.eps = codebooks, bool(normalize), float(eps)
        from ._lib import nonblocking_stream
        self._decode_stream = nonblocking_stream(codebooks.device)   # no implicit sync with the default stream
        self._pending = None

    def push(self, render_fn) -> torch.Tensor | None:
        """Render one view on the caller's current stream (render_fn returns its
        (L*K, H, W) weight map) and queue its decode; returns the previous
        view's features, or None for the first view."""
        with torch.no_grad():
            wm = render_fn()
        cur = torch.cuda.current_stream(wm.device)
        rendered = torch.cuda.Event()
        rendered.record(cur)
        prev = self._take(cur)   # the caller's stream waits for the previous decode only now
        # the output is allocated on the caller's stream (where it is used and freed) and
        # kept from reuse until the decode stream has written it
        L, _, Df = self.codebooks.shape
        out = torch.empty((L, Df) + tuple(wm.shape[1:]), dtype=torch.float32, device=wm.device)
        with torch.cuda.stream(self._decode_stream):
            self._decode_stream.wait_event(rendered)
            decode_language_features(wm, self.codebooks, self.normalize, self.eps, out=out)
            decoded = torch.cuda.Event()
            decoded.record(self._decode_stream)
        wm.record_stream(self._decode_stream)    # the map stays allocated until its decode ran
        out.record_stream(self._decode_stream)
        self._pending = (out, decoded)
        return prev

    def flush(self) -> torch.Tensor | None:
        """The last pushed view's features (None if there is none pending)."""
        return self._take(torch.cuda.current_stream(self.codebooks.device))

    def _take(self, cur):
        if self._pending is None:
            return None
        out, decoded = self._pending
        self._pending = None
        cur.wait_event(decoded)
        return out


def compute_final_feature_map(weight_map: torch.Tensor, codebooks: torch.Tensor) -> torch.Tensor:
    """scene/gaussian_model.py:545-550: codebooks.view(-1, Df).T @ weight_map.view(R, -1) -> (Df, H, W)
    for any number of levels / codes R = codebooks.numel() // Df (the reference accepts any R).  The
    codes are decoded in 64-code blocks on the matrix cores (R padded with zero codes to a multiple of
    64) and the per-block maps summed."""
    Df = codebooks.shape[-1]
    cb = codebooks.reshape(-1, Df)
    R = cb.shape[0]
    if weight_map.dim() != 3 or weight_map.shape[0] != R:
        raise ValueError(f"compute_final_feature_map: weight_map must be ({R}, H, W), got {tuple(weight_map.shape)}")
    Rp = (R + 63) // 64 * 64
    wm = weight_map
    if Rp != R:
        cb = torch.cat([cb, cb.new_zeros((Rp - R, Df))], 0)
        wm = torch.cat([wm, wm.new_zeros((Rp - R,) + tuple(wm.shape[1:]))], 0)
    out = decode_language_features(wm, cb.reshape(Rp // 64, 64, Df), normalize=False)
    return out[0] if out.shape[0] == 1 else out.sum(0)
