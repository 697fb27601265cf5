"""Host-side cost of one rasterizer forward at cfg2 (100K Gaussians, 800x800):
wall time per call with the GPU far ahead / behind, and a cProfile of 200 calls."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
from langsplatv2_amd.scenes import CONFIGS, make_camera, make_gaussians  # noqa: E402
import bench  # noqa: E402

cfg = CONFIGS[int(os.environ.get("LSR_CFG", "2"))]
dev = torch.device("cuda:0")
cam = make_camera(cfg["W"], cfg["H"])
g = {k: v.to(dev) for k, v in make_gaussians(cfg["N"], cam, seed=0, sh_degree=3, lang_dim=cfg["lang_dim"]).items()
     if isinstance(v, torch.Tensor)}
r = GaussianRasterizer(bench.settings(cam, dev, 3, cfg["lang_dim"] > 0))
z = torch.zeros_like(g["means3D"])


def fwd():
    with torch.no_grad():
        return r(means3D=g["means3D"], means2D=z, opacities=g["opacities"], shs=g["shs"],
                 language_feature_precomp=g.get("language_feature_precomp"), scales=g["scales"],
                 rotations=g["rotations"])


for _ in range(20):
    fwd()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(200):
    fwd()
torch.cuda.synchronize()
print(f"per forward {1e6 * (time.perf_counter() - t) / 200:.1f} us")
pr = cProfile.Profile()
pr.enable()
for _ in range(200):
    fwd()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
