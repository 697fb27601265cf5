"""langsplatv2_amd — MI355X-native (gfx950 HIP) differentiable tile rasterizer
for high-dimensional language Gaussian splatting.

The drop-in operator surface lives in `diff_gaussian_rasterization` (a thin
top-level package re-exporting `langsplatv2_amd.rasterizer`), so LangSplatV2's
gaussian_renderer/__init__.py and train.py run unchanged.  Compute is in
liblsr.so (C ABI: include/lsr.h).
"""
from ._lib import deterministic, set_deterministic  # noqa: F401
from .rasterizer import (GaussianRasterizationSettings, GaussianRasterizer,  # noqa: F401
                         rasterize_gaussians)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "deterministic",
           "set_deterministic"]
