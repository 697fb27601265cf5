"""`simple_knn._C` surface: distCUDA2 (see langsplatv2_amd/knn.py)."""
from langsplatv2_amd.knn import distCUDA2  # noqa: F401

__all__ = ["distCUDA2"]
