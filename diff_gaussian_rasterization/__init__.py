"""Drop-in replacement for the reference's `diff_gaussian_rasterization`
package (imported at gaussian_renderer/__init__.py:15), backed by the
MI355X-native HIP rasterizer in langsplatv2_amd (liblsr.so)."""
from langsplatv2_amd.rasterizer import (GaussianRasterizationSettings, GaussianRasterizer,  # noqa: F401
                                        rasterize_gaussians)

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians"]
