"""Fused Adam for the reference's optimizer.

The reference builds `torch.optim.Adam(l, lr=0.0, eps=1e-15)` over named
parameter groups (scene/gaussian_model.py:234-255) — in feature mode the
(N, 64) language logits and the (layers, 64, 512) codebooks, stepped once per
`accum_iter` iterations (train.py:261-263).  torch's default (foreach)
implementation makes ~7 elementwise passes per tensor; `FusedAdam` does the
same update in one HIP pass per tensor (csrc/adam.hip, C ABI lsr_adam_step).

It is a drop-in: same constructor arguments, `param_groups` with the
reference's extra keys ("name"), and the per-parameter state keys
"step" / "exp_avg" / "exp_avg_sq" that the reference's densification code
rewrites in place (replace_tensor_to_optimizer, _prune_optimizer,
cat_tensors_to_optimizer: scene/gaussian_model.py:352-420).  amsgrad and
maximize are not supported (the reference uses neither); there is no CPU path.
"""
from __future__ import annotations

import torch

from . import _lib
from .rasterizer import _stream


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("FusedAdam: invalid lr / eps / betas")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda or p.dtype != torch.float32:
                    raise RuntimeError("FusedAdam: parameters must be fp32 ROCm device tensors (there is no CPU path)")
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam: sparse gradients are not supported")
                if not p.is_contiguous():
                    raise RuntimeError("FusedAdam: parameters must be contiguous")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                state["step"] += 1
                g = p.grad.contiguous()
                m, v = state["exp_avg"], state["exp_avg_sq"]
                _lib.check(lib.lsr_adam_step(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                                             float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                                             float(group["weight_decay"]), int(state["step"].item()),
                                             _stream(p.device)), "lsr_adam_step")
                # the kernel wrote p, m and v through raw pointers: bump their
                # version counters as an in-place torch op would, so caches keyed
                # on _version (quick.decode_plan) and autograd's saved-tensor
                # checks see the update
                torch.autograd.graph.increment_version((p, m, v))
        return loss
