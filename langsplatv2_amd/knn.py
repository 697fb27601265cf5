"""simple_knn._C.distCUDA2 on the MI355X (csrc/knn.hip, C ABI lsr_knn_dist2).

Called once per scene by GaussianModel.create_from_pcd
(scene/gaussian_model.py:20,194): dist2 = clamp_min(distCUDA2(points), 1e-7)
becomes the initial log-scales.  Returns, for points (N, 3) fp32 on the
device, the mean of the three smallest squared distances to the other
points (exact; bit-identical to the brute-force oracle).  There is no CPU
path.
"""
from __future__ import annotations

import torch

from . import _lib
from .rasterizer import _Alloc, _stream


def distCUDA2(points: torch.Tensor) -> torch.Tensor:  # noqa: N802 (reference name)
    if points.dim() != 2 or points.shape[1] != 3:
        raise ValueError(f"distCUDA2: points must be (N, 3), got {tuple(points.shape)}")
    if not points.is_cuda:
        raise RuntimeError("distCUDA2: points must be a ROCm device tensor (there is no CPU path)")
    p = points.contiguous().float()
    out = torch.empty((p.shape[0],), dtype=torch.float32, device=p.device)
    alloc = _Alloc(p.device)
    _lib.check(_lib.load().lsr_knn_dist2(p.data_ptr(), p.shape[0], out.data_ptr(), alloc.fn, None,
                                         _stream(p.device)), "distCUDA2")
    return out
