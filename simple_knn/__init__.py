"""Drop-in replacement for the reference's `simple_knn` submodule
(`from simple_knn._C import distCUDA2`, scene/gaussian_model.py:20), backed
by the MI355X-native HIP kernel in langsplatv2_amd (liblsr.so)."""
